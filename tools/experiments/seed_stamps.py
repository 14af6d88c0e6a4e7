"""Lab: phase clocks of the MFMA seed blocks at c1 (1000 x 10000 x 256 dot,
k = 10).  Needs PMM_LIB=libpmm_st.so (make ab AB=-DPMM_SEED_STAMPS
AB_NAME=libpmm_st.so).  Prints, over the seed blocks of the last call, the
median and max of each phase (s_memtime ticks) and the spread of the blocks'
start times; the prologue's event time alongside."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, "polars-matmul_amd")
from polars_matmul import _native as nat  # noqa: E402

L = nat.lib()
m, n, d, k = 1000, 10000, 256, 10
metric = nat.metric_from_str(sys.argv[1] if len(sys.argv) > 1 else "dot")
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.randn(m, d, device="cuda", generator=g)
c = torch.randn(n, d, device="cuda", generator=g)
oi = torch.empty(m, k, dtype=torch.int32, device="cuda")
osc = torch.empty(m, k, device="cuda")
nat.timing_enable(True)
for it in range(30):
    if it == 10:
        nat.timing_reset()
    nat.topk_device(q.data_ptr(), d, m, c.data_ptr(), d, n, d, k, metric, oi.data_ptr(), osc.data_ptr())
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (1024 * 8))()
assert L.pmm_lab_seed_stamps(buf, 1024) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8).astype(np.int64)
nb = (m + 15) // 16
a = a[:nb]
names = ["stage q + chunk 0", "K loop", "norms", "keys", "selection"]
for i, nm in enumerate(names):
    dlt = a[: nb - 1, i + 1] - a[: nb - 1, i]
    print(f"{nm:20s} median {int(np.median(dlt)):7d}  max {int(dlt.max()):7d}")
tot = a[: nb - 1, 5] - a[: nb - 1, 0]
print(f"{'block total':20s} median {int(np.median(tot)):7d}  max {int(tot.max()):7d}")
print(f"block start spread {int(a[:, 0].max() - a[:, 0].min())}, first start -> last end {int(a[: nb - 1, 5].max() - a[:, 0].min())}")
for kname in ("gemm_f32_seed", "gemm_f32_fused", "merge"):
    try:
        print(kname, nat.timing_read(kname))
    except Exception as e:  # noqa: BLE001
        print(kname, "n/a", e)
