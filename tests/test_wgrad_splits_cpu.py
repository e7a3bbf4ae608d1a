"""Row-split choice of the own dense weight-gradient kernel (fused_dense._w4w_splits):
splits x 256^2-tiles <= 256 (one tile per CU), >= 1024 rows and whole 64-row K-tiles per
split."""
from apex_example_amd import fused_dense as FD


def test_w4w_splits_bert_and_gpt2_shapes():
    assert FD._w4w_splits(16384, 4096, 1024) == 4      # 64 tiles
    assert FD._w4w_splits(16384, 3072, 1024) == 4      # 48 tiles (8 would be 384 > 256)
    assert FD._w4w_splits(16384, 1024, 1024) == 16     # 16 tiles
    assert FD._w4w_splits(8192, 1024, 1024) == 8       # >= 1024 rows per split
    assert FD._w4w_splits(2048, 256, 256) == 2


def test_w4w_splits_invariants():
    for T in (64, 1000, 1024, 3072, 8192, 16384, 24576):
        for o, i in ((256, 256), (1024, 4096), (4096, 4096), (768, 3072)):
            S = FD._w4w_splits(T, o, i)
            tiles = (o // 256) * (i // 256)
            assert S >= 1 and (S == 1 or (S * tiles <= 256 and T % (S * 64) == 0
                                          and T // S >= 1024))


def test_w4w_splits_side_stream_cap():
    """On the weight-gradient side stream the grid is capped (128 workgroups by default)."""
    assert FD._w4w_splits(8192, 4096, 1024, 128) == 2
    assert FD._w4w_splits(16384, 3072, 1024, 128) == 2
    assert FD._w4w_splits(16384, 4096, 1024, 64) == 1
