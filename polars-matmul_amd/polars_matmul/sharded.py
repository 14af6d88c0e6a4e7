"""Corpus-row-sharded top-k across the GPUs of one node.

One process per GPU (``torch.distributed``; backend "nccl" is RCCL on ROCm).
Every rank holds the full query block and a contiguous slice of the corpus
rows; it runs the fused top-k on its slice with ``index_base`` = the slice's
first global row, so its list already carries global corpus indices.  Rank 0
gathers the per-rank ``M x k`` (index, score) lists over RCCL (xGMI) -- one
collective, both planes of every rank landing in one ``[world][2][M][k]``
buffer -- and k-way merges them in place.  The gather is the path's only exchange step; there is no
collective on the GEMM itself.

The reference is single-process (no counterpart).  The local top-k and the
merge are injectable so the orchestration (partitioning, index bases, gather
layout, merge) is exercised on CPU with the gloo backend in tests; on MI355X
the defaults call libpmm (``pmm_topk_f32_device`` / ``pmm_merge_topk_device``).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous corpus rows [lo, hi) owned by `rank` (sizes differ by <= 1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    return n * rank // world, n * (rank + 1) // world


def zero_padded(t: torch.Tensor, align: int = 32) -> torch.Tensor:
    """A (rows, d) view whose row stride is roundup(d, align) with zero-filled
    padding columns, as pmm_topk_f32_device (align 32) and
    pmm_topk_bf16_device (align 128) require (include/pmm.h)."""
    rows, d = t.shape
    dp = -(-d // align) * align
    if d == dp and t.is_contiguous():
        return t
    buf = torch.zeros((rows, dp), dtype=t.dtype, device=t.device)
    buf[:, :d] = t
    return buf[:, :d]


def _device_topk(q: torch.Tensor, c: torch.Tensor, k: int, metric: int, index_base: int,
                 out_i: torch.Tensor, out_s: torch.Tensor, workspace: Optional[torch.Tensor]) -> None:
    from . import _native

    m, d = q.shape
    n = c.shape[0]
    ws_ptr = workspace.data_ptr() if workspace is not None else 0
    ws_bytes = workspace.numel() if workspace is not None else 0
    _native.topk_device(q.data_ptr(), q.stride(0), m, c.data_ptr(), c.stride(0), n, d, k, metric,
                        out_i.data_ptr(), out_s.data_ptr(), index_base=index_base,
                        workspace=ws_ptr, workspace_bytes=ws_bytes,
                        stream=torch.cuda.current_stream(q.device).cuda_stream)


def _device_topk_bf16(q: torch.Tensor, c: torch.Tensor, k: int, metric: int, index_base: int,
                      out_i: torch.Tensor, out_s: torch.Tensor, workspace: Optional[torch.Tensor]) -> None:
    from . import _native

    m, d = q.shape
    n = c.shape[0]
    ws_ptr = workspace.data_ptr() if workspace is not None else 0
    ws_bytes = workspace.numel() if workspace is not None else 0
    _native.topk_bf16_device(q.data_ptr(), q.stride(0), m, c.data_ptr(), c.stride(0), n, d, k, metric,
                             out_i.data_ptr(), out_s.data_ptr(), index_base=index_base,
                             workspace=ws_ptr, workspace_bytes=ws_bytes,
                             stream=torch.cuda.current_stream(q.device).cuda_stream)


def _device_merge(gathered: torch.Tensor, k: int, metric: int, out_i: torch.Tensor,
                  out_s: torch.Tensor) -> None:
    """k-way merge of the gathered [world][2][M][k_in] lists (per rank: an
    index plane, then a score plane) in place, with no re-layout copy
    (pmm_merge_sorted_topk_strided_device: every rank's lists are its top-k,
    best first, so each row reads only the prefixes that can hold its answer)."""
    from . import _native

    world, _, m, kin = gathered.shape
    _native.merge_strided_device(gathered.data_ptr(), gathered[0, 1].data_ptr(), m, world, kin,
                                 kin, 2 * m * kin, k, metric, out_i.data_ptr(), out_s.data_ptr(),
                                 stream=torch.cuda.current_stream(gathered.device).cuda_stream,
                                 sorted_lists=True)


class ShardedTopK:
    """Reusable per-rank state for repeated sharded top-k passes.

    queries: (M, D) f32 tensor (replicated on every rank), or bf16 for the
        bf16 compute path (pmm_topk_bf16_device)
    corpus_shard: (n_local, D) tensor of the same dtype, rows
        [index_base, index_base + n_local)
    Returns from ``run()``: (idx int32 (M, k), score f32 (M, k)) on rank 0 (the
    global top-k), the local lists on other ranks.
    """

    def __init__(self, queries: torch.Tensor, corpus_shard: torch.Tensor, index_base: int, k: int,
                 metric: int, group=None,
                 local_topk: Optional[Callable] = None, merge: Optional[Callable] = None,
                 workspace: Optional[torch.Tensor] = None):
        if local_topk is None:
            bf16 = queries.dtype == torch.bfloat16
            align = 128 if bf16 else 32
            queries, corpus_shard = zero_padded(queries, align), zero_padded(corpus_shard, align)
            local_topk = _device_topk_bf16 if bf16 else _device_topk
        self.q = queries
        self.c = corpus_shard
        self.index_base = int(index_base)
        self.k = int(k)
        self.metric = int(metric)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.local_topk = local_topk or _device_topk
        self.merge = merge or _device_merge
        self.workspace = workspace
        m = queries.shape[0]
        dev = queries.device
        # this rank's list as one [2][M][k] block of 32-bit words (index plane,
        # score plane), so ONE gather moves both into the root's
        # [world][2][M][k] buffer, which the merge reads in place
        self.loc = torch.empty((2, m, self.k), dtype=torch.int32, device=dev)
        self.loc_i = self.loc[0]
        self.loc_s = self.loc[1].view(torch.float32)
        if self.world > 1 and self.rank == 0:
            self.gathered = torch.empty((self.world, 2, m, self.k), dtype=torch.int32, device=dev)
            self._gather_list = list(self.gathered.unbind(0))
            self.out_i = torch.empty_like(self.loc_i)
            self.out_s = torch.empty_like(self.loc_s)

    def run(self) -> Tuple[torch.Tensor, torch.Tensor]:
        self.local_topk(self.q, self.c, self.k, self.metric, self.index_base,
                        self.loc_i, self.loc_s, self.workspace)
        if self.world == 1:
            return self.loc_i, self.loc_s
        root = self.rank == 0
        dist.gather(self.loc, self._gather_list if root else None, dst=0, group=self.group)
        if not root:
            return self.loc_i, self.loc_s
        self.merge(self.gathered, self.k, self.metric, self.out_i, self.out_s)
        return self.out_i, self.out_s
