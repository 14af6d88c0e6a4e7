"""Merge kernel debugging aid: random per-list (index, score) inputs through
pmm_merge_topk_device, compared with a NumPy merge; run once per
PMM_MERGE_REG value (read once per process)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "polars-matmul_amd"))
from polars_matmul import _native as n  # noqa: E402


def case(m, s, k_in, k_out, seed=0):
    rs = np.random.RandomState(seed)
    idx = np.stack([rs.permutation(100000)[: s * k_in] for _ in range(m)]).reshape(m, s, k_in).astype(np.uint32)
    sc = rs.rand(m, s, k_in).astype(np.float32)
    dev = torch.device("cuda:0")
    ti = torch.from_numpy(idx.view(np.int32)).to(dev)
    ts = torch.from_numpy(sc).to(dev)
    oi = torch.empty(m, k_out, dtype=torch.int32, device=dev)
    os_ = torch.empty(m, k_out, dtype=torch.float32, device=dev)
    n.merge_device(ti.data_ptr(), ts.data_ptr(), m, s, k_in, k_out, 1, oi.data_ptr(), os_.data_ptr())
    torch.cuda.synchronize()
    gi = oi.cpu().numpy().view(np.uint32)
    gs = os_.cpu().numpy()
    bad = 0
    for r in range(m):
        fi, fs = idx[r].ravel(), sc[r].ravel()
        order = np.lexsort((fi, -fs))[:k_out]
        if not (np.array_equal(gi[r], fi[order]) and np.array_equal(gs[r], fs[order])):
            if bad < 2:
                print(f"row {r}: got {gi[r][:8]} {gs[r][:8]}\n        want {fi[order][:8]} {fs[order][:8]}")
            bad += 1
    print(f"m={m} s={s} k_in={k_in} k_out={k_out}: {bad} bad rows")


if __name__ == "__main__":
    for args in [(4, 3, 50, 20), (4, 1, 30, 20), (8, 8, 100, 100), (8, 16, 128, 128), (8, 2, 700, 100)]:
        case(*args)
