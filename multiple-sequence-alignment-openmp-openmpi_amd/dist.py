"""Multi-GPU layer: one process per GPU, pairs sharded, one all-gather.

Replaces the reference's MPI master/worker queue (submit/xuliny-seqalkway.cpp:
272-361 master, 369-417 workers, Packet records 126-152): the m*n cost of
every pair is known up front, so each rank takes a static LPT cell-cost shard
(seqalign.shard_pairs), aligns it on its own GPU, and the fixed-size 72-byte
result records {int32 pair_id, int32 penalty, uint8 problemhash[64]} of all
ranks are collected with ONE all_gather_into_tensor (backend "nccl" = RCCL
over xGMI on MI355X; "gloo" in the CPU tests).  Every rank then holds the
penalties and problem hashes in canonical order; rank 0 runs the sequential
hash chain (sub:334-337).

Failure contract (the C++ in-process path tags records the same way): a rank
whose alignment raises still contributes its block, every record tagged
FAILED, to the one collective; every rank then raises RankFailed instead of
some ranks hanging in the all-gather.
"""
import numpy as np
import torch
import torch.distributed as dist

import seqalign

REC = 72


def shard_sizes(lengths, world):
    return [len(seqalign.shard_pairs(lengths, r, world)) for r in range(world)]


def pack_records(ids, penalties, hashes, per):
    rec = np.zeros((per, REC), dtype=np.uint8)
    head = np.full((per, 2), -1, dtype=np.int32)
    n = len(ids)
    head[:n, 0] = np.asarray(ids, dtype=np.int32)
    head[:n, 1] = np.asarray(penalties, dtype=np.int32)
    rec[:, :8] = head.view(np.uint8).reshape(per, 8)
    if n:
        rec[:n, 8:] = np.asarray(hashes, dtype=np.uint8).reshape(n, 64)
    return rec


FAILED = -2  # pair_id of every record of a rank whose alignment failed


class RankFailed(RuntimeError):
    pass


def unpack_records(gathered, P):
    """Canonical-order penalties int32[P] and raw hashes uint8[P,64].
    Raises RankFailed on every rank when some rank contributed FAILED records."""
    g = np.ascontiguousarray(gathered, dtype=np.uint8).reshape(-1, REC)
    head = g[:, :8].copy().view(np.int32).reshape(-1, 2)
    if (head[:, 0] == FAILED).any():
        per = g.shape[0]
        bad = sorted({r for r in range(per) if head[r, 0] == FAILED})
        raise RankFailed("all-gather: a rank failed to align its shard (records %d..%d tagged %d)"
                         % (bad[0], bad[-1], FAILED))
    pen = np.zeros(P, dtype=np.int32)
    hs = np.zeros((P, 64), dtype=np.uint8)
    seen = np.zeros(P, dtype=bool)
    for r in range(g.shape[0]):
        pid = int(head[r, 0])
        if pid < 0:
            continue
        if pid >= P or seen[pid]:
            raise RuntimeError("all-gather: bad or duplicate pair id %d" % pid)
        seen[pid] = True
        pen[pid] = head[r, 1]
        hs[pid] = g[r, 8:]
    if not seen.all():
        raise RuntimeError("all-gather: %d pairs missing" % int((~seen).sum()))
    return pen, hs


def all_gather_records(rec, device=None, group=None):
    """ONE collective: every rank contributes `per` records."""
    world = dist.get_world_size(group)
    t = torch.from_numpy(rec)
    if device is not None:
        t = t.to(device, non_blocking=False)
    out = torch.empty((world * rec.shape[0], REC), dtype=torch.uint8, device=t.device)
    dist.all_gather_into_tensor(out, t, group=group)
    return out.cpu().numpy()


def align_sharded(align_fn, lengths, pxy, pgap, rank, world, device=None, group=None):
    """Runs this rank's shard through align_fn(ids, pxy, pgap) -> (pen, hashes),
    gathers every rank's records and returns (penalties[P], hashes[P,64], ids)."""
    k = len(lengths)
    P = k * (k - 1) // 2
    ids = seqalign.shard_pairs(lengths, rank, world)
    per = max(shard_sizes(lengths, world) + [1])
    err = None
    try:
        pen, hs = align_fn(ids, pxy, pgap)
        rec = pack_records(ids, pen, hs, per)
    except Exception as e:  # still join the ONE collective, so no peer waits forever
        err = e
        rec = pack_records([], [], [], per)
        rec[:, :4] = np.array([FAILED], dtype=np.int32).view(np.uint8)
    g = all_gather_records(rec, device=device, group=group)
    if err is not None:
        raise RankFailed("rank %d: %s" % (rank, err)) from err
    pen_all, hs_all = unpack_records(g, P)
    return pen_all, hs_all, ids
