"""Compare the r64 and ws bf16 kernels on a few cases and print the first
mismatching rows (debugging aid)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "polars-matmul_amd"))
from polars_matmul import _native as n  # noqa: E402

METRICS = {"cosine": 0, "dot": 1, "euclidean": 2}


def run(q, c, k, metric, r64):
    os.environ["PMM_BF16_R64"] = r64
    return n.topk_host(q, c, k, METRICS[metric], compute=n.COMPUTE_BF16)


def case(m, nn, d, k, metric, env=None, seed=0):
    env = env or {}
    old = {key: os.environ.get(key) for key in env}
    os.environ.update(env)
    rs = np.random.RandomState(m + nn + d + k + 11 + seed)
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(nn, d).astype(np.float32)
    ri, rsc = run(q, c, k, metric, "1")
    wi, wsc = run(q, c, k, metric, "0")
    for key, v in old.items():
        if v is None:
            os.environ.pop(key, None)
        else:
            os.environ[key] = v
    bad = np.nonzero((ri != wi).any(axis=1))[0]
    print(f"{m}x{nn}x{d} k={k} {metric} {env}: mismatching rows {len(bad)} {bad[:10]}", flush=True)
    for r in bad[:2]:
        j = np.nonzero(ri[r] != wi[r])[0]
        print("  row", r, "diff at", j[:4], "r64", ri[r][j[:4]], rsc[r][j[:4]], "ws", wi[r][j[:4]], wsc[r][j[:4]], flush=True)
        # where does the ws top index land in r64's list, with which score?
        for col in wi[r][j[:2]]:
            pos = np.nonzero(ri[r] == col)[0]
            qb = q[r].astype(np.float64)
            cb = c[col].astype(np.float64)
            # bf16 rounding (RNE) of the inputs, as the kernels see them
            def bf(x):
                u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
                u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
                return u.astype(np.uint32).view(np.float32).astype(np.float64)
            qb, cb = bf(q[r]), bf(c[col])
            tru = qb @ cb / (np.linalg.norm(qb) * np.linalg.norm(cb)) if metric == "cosine" else qb @ cb
            print("   ws col", col, "tile", col // 32, "in r64 at", pos, rsc[r][pos] if len(pos) else None,
                  "truth", tru, flush=True)


if __name__ == "__main__":
    case(33, 70000, 128, 50, "cosine")
    case(33, 70000, 128, 50, "euclidean")
    case(33, 70000, 128, 50, "cosine", {"PMM_BF16_SEED": "0"})
    case(64, 70000, 128, 50, "cosine")
    case(300, 70000, 128, 50, "cosine")
    case(33, 70000, 128, 50, "dot")
    case(33, 70000, 256, 50, "cosine", seed=1)
    case(33, 200000, 256, 50, "cosine")
    case(33, 70000, 128, 10, "cosine")
