"""FLOP / byte estimates from an op signature string (apex.pyprof.prof's per-op
models, reduced to the ops that dominate training steps)."""
from __future__ import annotations

import re

_BYTES = {"float32": 4, "float": 4, "float16": 2, "half": 2, "bfloat16": 2, "float64": 8,
          "int64": 8, "int32": 4, "int8": 1, "uint8": 1, "bool": 1}


def parse_signature(sig):
    """'linear(8x1024 bfloat16, 4096x1024 bfloat16)' -> ('linear', [((8,1024),'bfloat16'), ...])"""
    m = re.match(r"^([^(]+)\((.*)\)$", sig.strip())
    if not m:
        return sig, []
    name, body = m.group(1), m.group(2)
    shapes = []
    for tok in re.findall(r"(?:^|, )(?:\w+=)?([0-9x]+|scalar) (\w+)", body):
        dims = () if tok[0] == "scalar" else tuple(int(d) for d in tok[0].split("x"))
        shapes.append((dims, tok[1]))
    return name, shapes


def _numel(d):
    n = 1
    for s in d:
        n *= s
    return n


def op_flops(sig):
    """Return (flops, bytes) for a signature, or (None, bytes) when unmodelled."""
    name, shapes = parse_signature(sig)
    nbytes = sum(_numel(d) * _BYTES.get(t, 4) for d, t in shapes)
    if not shapes:
        return None, 0
    try:
        if name in ("linear",) and len(shapes) >= 2:
            x, w = shapes[0][0], shapes[1][0]
            return 2 * _numel(x[:-1]) * w[0] * w[1], nbytes
        if name in ("matmul", "mm", "bmm", "__matmul__") and len(shapes) >= 2:
            a, b = shapes[0][0], shapes[1][0]
            batch = _numel(a[:-2]) if len(a) > 2 else 1
            return 2 * batch * a[-2] * a[-1] * b[-1], nbytes
        if name in ("addmm",) and len(shapes) >= 3:
            a, b = shapes[1][0], shapes[2][0]
            return 2 * a[0] * a[1] * b[1], nbytes
        if name in ("conv2d",) and len(shapes) >= 2:
            x, w = shapes[0][0], shapes[1][0]
            # stride/padding not in the signature: assume 'same' output size
            n, _, h, wd = x
            return 2 * n * h * wd * w[0] * w[1] * w[2] * w[3], nbytes
        if name == "scaled_dot_product_attention" and len(shapes) >= 3:
            q, k = shapes[0][0], shapes[1][0]
            return 4 * _numel(q[:-2]) * q[-2] * k[-2] * q[-1], nbytes
    except (IndexError, ValueError):
        pass
    return None, nbytes
