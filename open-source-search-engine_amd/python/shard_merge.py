"""Msg39 -> Msg3a exchange for docid-range shards.

Every rank holds one docid range of every termlist and produces its own top
list; the lists are all-gathered (RCCL on the GPU box, gloo in the CPU tests)
and every rank merges them the way Msg3a::mergeLists does (Msg3a.cpp:1315-
1467, via gbgpu_merge_topk).  Hit counts are summed (Msg3a.cpp:1588-1615 sums
the shards' m_docIdVoteBuf counts)."""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

import gbgpu


def gather_merge(docids: np.ndarray, scores: np.ndarray, hits: int, k: int, device: str = "cuda"):
    """Returns (total hits, merged docids, merged scores as float64)."""
    world = dist.get_world_size()
    n = min(len(docids), k)
    # one record per slot: (docid, score) as float64 (docids are 38-bit: exact)
    rec = torch.zeros((k, 2), dtype=torch.float64, device=device)
    if n:
        rec[:n, 0] = torch.from_numpy(np.asarray(docids[:n], dtype=np.float64)).to(device)
        rec[:n, 1] = torch.from_numpy(np.asarray(scores[:n], dtype=np.float64)).to(device)
    cnt = torch.tensor([n, hits], dtype=torch.int64, device=device)
    recs = [torch.empty_like(rec) for _ in range(world)]
    cnts = [torch.empty_like(cnt) for _ in range(world)]
    dist.all_gather(recs, rec)
    dist.all_gather(cnts, cnt)
    shards = []
    total = 0
    for r, c in zip(recs, cnts):
        r, c = r.cpu().numpy(), c.cpu().numpy()
        m = int(c[0])
        total += int(c[1])
        shards.append((r[:m, 0].astype(np.int64), r[:m, 1].astype(np.float32)))
    d, s = gbgpu.merge_topk(shards, k)
    return total, d, s
