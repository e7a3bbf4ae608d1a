"""Reference-parity driver (examples/spawn_train.py) end-to-end on CPU: two
gloo workers via mp.spawn, amp + apex-style DDP and the torch-DDP path, plus
the fault-injection switch and the metrics logger."""
import json
import os
import subprocess
import sys

import pytest
import torch

import dist_workers as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_example(tmp_path, *extra):
    out = tmp_path / "res.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(W.free_port()),
               CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, os.path.join(ROOT, "examples", "spawn_train.py"), "--cpu",
           "--gpus", "2", "--epochs", "2", "--dataset_size", "800", "--batch_size", "40",
           "--lr", "0.05", "--log_every", "5", "--result_file", str(out), *extra]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    return json.loads(out.read_text()), p.stdout


@pytest.mark.parametrize("extra", [("--apex_opt_level", "O2"), ("--apex_opt_level", "O0"),
                                   ("--apex_enabled", "false")])
def test_spawn_train_learns(tmp_path, extra):
    res, stdout = _run_example(tmp_path, *extra)
    assert res["world_size"] == 2 and res["steps_per_epoch"] == 10
    assert res["final_loss"] < res["first_loss"] * 0.7, res
    assert "Epoch [2/2], Step [10/10], Loss:" in stdout
    assert "Training complete in:" in stdout


def test_str2bool():
    from apex_example_amd.utils.data import str2bool

    assert str2bool("False") is False and str2bool("0") is False and str2bool("yes") is True
    with pytest.raises(Exception):
        str2bool("maybe")


def test_synthetic_mnist_contract():
    from apex_example_amd.utils.data import SyntheticMNIST

    ds = SyntheticMNIST(n=100)
    x, y = ds[3]
    assert x.shape == (1, 28, 28) and x.dtype == torch.float32
    assert 0.0 <= float(x.min()) and float(x.max()) <= 1.0 and 0 <= y < 10
    x2, _ = ds[3]
    assert torch.equal(x, x2)  # deterministic per index


def test_fault_injection_drives_overflow_skip():
    from apex_example_amd import amp
    from apex_example_amd.optimizers import FusedSGD
    from apex_example_amd.utils import fault

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.ReLU(), torch.nn.Linear(8, 2))
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9)
    model, opt = amp.initialize(model, opt, opt_level="O2", half_dtype=torch.bfloat16,
                                verbosity=0)
    fault.configure("nan@step=2,param=1")
    try:
        x = torch.randn(4, 8)
        y = torch.randint(0, 2, (4,))
        scales = []
        for it in range(4):
            before = [p.detach().clone() for p in amp.master_params(opt)]
            loss = torch.nn.functional.cross_entropy(model(x).float(), y)
            opt.zero_grad()
            with amp.scale_loss(loss, opt) as s:
                s.backward()
            opt.step()
            scales.append(amp.state_dict()["loss_scaler0"]["loss_scale"])
            unchanged = all(torch.equal(a, b) for a, b in zip(before, amp.master_params(opt)))
            assert unchanged == (it == 2)
        assert fault.fired() == 1
        assert scales[2] == scales[1] / 2
    finally:
        fault.disable()


def test_fault_spec_parse():
    from apex_example_amd.utils.fault import parse

    s = parse("inf@step=3,rank=1,param=4,every=5")
    assert (s.step, s.rank, s.param, s.every) == (3, 1, 4, 5) and s.value == float("inf")
    assert s.fires(8, 1) and not s.fires(8, 0) and not s.fires(4, 1)
    with pytest.raises(ValueError):
        parse("inf@rank=1")


def test_metrics_logger(tmp_path):
    from apex_example_amd.utils.metrics import MetricsLogger

    path = tmp_path / "m.jsonl"
    log = MetricsLogger(every=3, units_per_step=32, unit="images", path=str(path), stream=None,
                        extra={"model": "x"})
    for i in range(7):
        log.update(loss=torch.tensor(1.0 / (i + 1)))
    recs = [json.loads(line) for line in path.read_text().splitlines()]
    assert [r["step"] for r in recs] == [3, 6]
    assert recs[0]["unit"] == "images/s" and recs[0]["throughput"] > 0
    assert recs[1]["model"] == "x" and abs(recs[1]["loss"] - 1 / 6) < 1e-6


def test_bench_self_spawns_gpus_ranks():
    """`python bench.py --gpus N` without torchrun starts N rank processes itself
    (gloo on this CPU host) and every rank sees world size N."""
    env = dict(os.environ, APEX_AMD_FORCE_CPU="1", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3",
                        "--dry-run"], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert rec == {"dry_run": True, "n_gpus": 3, "backend": "gloo", "launcher": "self-spawn"}


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, APEX_AMD_FORCE_CPU="1", WORLD_SIZE="1", RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dry-run"], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 3
    assert "refusing" in p.stderr
