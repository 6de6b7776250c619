"""Generates tests/golden/local_reduce.npz from the CPU oracle (oracle/hccl_oracle.c).

The reference holds no numeric fixtures for this path (its ST verifier is symbolic), so the
fixtures are the oracle's output on: every ordered pair of edge values (±0 ties, NaN, ±Inf, subnormals,
extremes, wrap-around) plus 509 seeded random pairs, for every reduce dtype x op. The KATs the reference does
hold (examples/02_collectives/*/README_en.md sample outputs) are checked directly in tests/test_oracle.py.

Run: python tests/golden/make_golden.py   (rewrites the .npz; the file is committed)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402


def main():
    out = {}
    for dtype in O.REDUCE_DTYPES:
        name = O.DTYPE_NAMES[dtype]
        es, ed = O.edge_cross(dtype)
        rs = O.random_operands(dtype, 509, seed=0x5EED0000 + dtype, edge=False)
        rd = O.random_operands(dtype, 509, seed=0x5EED1000 + dtype, edge=False)
        src = np.ascontiguousarray(np.concatenate([es, rs]))
        dst = np.ascontiguousarray(np.concatenate([ed, rd]))
        out[f"{name}_src"] = src
        out[f"{name}_dst"] = dst
        for op in O.OPS:
            out[f"{name}_{O.OP_NAMES[op]}"] = O.local_reduce(dtype, op, dst.copy(), src)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "local_reduce.npz")
    np.savez_compressed(path, **out)
    print(path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
