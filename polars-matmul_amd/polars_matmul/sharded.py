"""Corpus-row-sharded top-k across the GPUs of one node.

One process per GPU (``torch.distributed``; backend "nccl" is RCCL on ROCm).
Every rank holds the full query block and a contiguous slice of the corpus
rows; it runs the fused top-k on its slice with ``index_base`` = the slice's
first global row, so its list already carries global corpus indices.  Rank 0
gathers the per-rank ``M x k`` (index, score) lists over RCCL (xGMI) and
k-way merges them.  The gather is the path's only exchange step; there is no
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


def _device_merge(lists_i: torch.Tensor, lists_s: torch.Tensor, k: int, metric: int,
                  out_i: torch.Tensor, out_s: torch.Tensor) -> None:
    from . import _native

    m, r, kin = lists_i.shape
    _native.merge_device(lists_i.data_ptr(), lists_s.data_ptr(), m, r, kin, k, metric,
                         out_i.data_ptr(), out_s.data_ptr(),
                         stream=torch.cuda.current_stream(lists_i.device).cuda_stream)


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
        self.loc_i = torch.empty((m, self.k), dtype=torch.int32, device=dev)
        self.loc_s = torch.empty((m, self.k), dtype=torch.float32, device=dev)
        if self.world > 1 and self.rank == 0:
            self.gath_i = [torch.empty_like(self.loc_i) for _ in range(self.world)]
            self.gath_s = [torch.empty_like(self.loc_s) for _ in range(self.world)]
            self.out_i = torch.empty_like(self.loc_i)
            self.out_s = torch.empty_like(self.loc_s)

    def run(self) -> Tuple[torch.Tensor, torch.Tensor]:
        self.local_topk(self.q, self.c, self.k, self.metric, self.index_base,
                        self.loc_i, self.loc_s, self.workspace)
        if self.world == 1:
            return self.loc_i, self.loc_s
        root = self.rank == 0
        dist.gather(self.loc_i, self.gath_i if root else None, dst=0, group=self.group)
        dist.gather(self.loc_s, self.gath_s if root else None, dst=0, group=self.group)
        if not root:
            return self.loc_i, self.loc_s
        lists_i = torch.stack(self.gath_i, dim=1).contiguous()  # [M][world][k]
        lists_s = torch.stack(self.gath_s, dim=1).contiguous()
        self.merge(lists_i, lists_s, self.k, self.metric, self.out_i, self.out_s)
        return self.out_i, self.out_s
