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


def unpack_chunk(gathered):
    """(ids, penalties, hashes) of the valid records of one chunk's all-gather.
    Raises RankFailed on every rank when some rank contributed FAILED records."""
    g = np.ascontiguousarray(gathered, dtype=np.uint8).reshape(-1, REC)
    head = g[:, :8].copy().view(np.int32).reshape(-1, 2)
    if (head[:, 0] == FAILED).any():
        raise RankFailed("all-gather: a rank failed to align its shard")
    ok = head[:, 0] >= 0
    return head[ok, 0].astype(np.int64), head[ok, 1].copy(), g[ok, 8:]


def chunk_parts(lengths, rank, world, chunks):
    """This rank's shard cut at global canonical thresholds P*c/chunks, and for
    every chunk the largest part over ranks (the padded record block size)."""
    k = len(lengths)
    P = k * (k - 1) // 2
    bounds = [P * c // chunks for c in range(chunks + 1)]
    cut = lambda ids, c: ids[(ids >= bounds[c]) & (ids < bounds[c + 1])]
    shards = [seqalign.shard_pairs(lengths, r, world) for r in range(world)]
    per = [max([len(cut(sh, c)) for sh in shards] + [1]) for c in range(chunks)]
    return [cut(shards[rank], c) for c in range(chunks)], per


def auto_chunks(P, world):
    """Pieces per rank: one.  A piece's pairs finish together at the end of its
    launch (strips: one wave per pair, one round), and a half-full launch takes
    as long as a full one, so two pieces cost a second fill: C4 at W = 8, 1
    piece 28.4 ms, 2 pieces 31.0 ms (profiles/r03/sched).
    align_sharded_pipelined keeps the piece machinery for chunks > 1."""
    return 1


def align_sharded_pipelined(eng, lengths, pxy, pgap, rank, world, chunks=1, device=None, group=None,
                            on_piece=None):
    """The shard in `chunks` pieces of ascending canonical ids: piece c+1 aligns
    on the GPU (Engine.align_pairs_begin) while piece c's records go through
    their all-gather and rank 0's chain worker (seqalign.ChainStream) advances
    over them -- sub:305-337 collects results as they arrive and then chains;
    here the chain of all but the last piece hides behind the alignment.
    Returns (hash on rank 0 else None, penalties[P], hashes[P,64]) on rank 0,
    (None, None, None) elsewhere.  Same failure contract as align_sharded:
    a failing rank joins every remaining collective with FAILED records."""
    k = len(lengths)
    P = k * (k - 1) // 2
    parts, per = chunk_parts(lengths, rank, world, chunks)
    chain = seqalign.ChainStream(P) if rank == 0 else None
    err = None       # this rank's failure, or a peer's seen in a gather
    pending = False  # an align_pairs_begin not yet ended
    try:
        try:
            eng.align_pairs_begin(parts[0], pxy, pgap)
            pending = True
        except Exception as e:
            err = e
        for c in range(chunks):
            rec = None
            if err is None:
                try:
                    pending = False
                    pen, hs = eng.align_pairs_end()
                    if on_piece is not None:
                        on_piece(c)
                    if c + 1 < chunks:
                        eng.align_pairs_begin(parts[c + 1], pxy, pgap)
                        pending = True
                    rec = pack_records(parts[c], pen, hs, per[c])
                except Exception as e:
                    err = e
            if rec is None:  # still join the collective, so no peer waits forever
                rec = pack_records([], [], [], per[c])
                rec[:, :4] = np.array([FAILED], dtype=np.int32).view(np.uint8)
            g = all_gather_records(rec, device=device, group=group)
            if err is not None:
                continue
            try:
                ids, pen, hs = unpack_chunk(g)
            except RankFailed as e:  # every rank sees it in the same gather
                err = e
                continue
            if chain is not None:
                chain.feed(ids, pen, hs)
        if err is not None:
            raise RankFailed("rank %d: %s" % (rank, err)) from err
        if chain is None:
            return None, None, None
        return chain.finish()
    finally:
        if pending:  # a peer failed while this rank's next piece was in flight
            try:
                eng.align_pairs_end()
            except Exception:
                pass
        if chain is not None:
            chain.close()


def align_sharded_streamed(eng, lengths, pxy, pgap, rank, world, chunks=8, device=None, group=None,
                           on_piece=None, poll_s=50e-6):
    """The shard as ONE launch (Engine.align_pairs_begin over its ids in
    ascending canonical order, the engine built with finalize="fused") whose
    per-pair records stream to the host as pairs are hashed inside the fill
    launch (Engine.align_pairs_poll).
    Piece c -- the shard's ids below the global threshold P (c+1) / chunks --
    goes through its all-gather as soon as all of its records are in, and rank
    0's chain worker advances over it while the rest of the shard still
    aligns: sub:305-331 collects results as they arrive, sub:334-337 chains.
    Same return value and failure contract as align_sharded_pipelined."""
    import time

    k = len(lengths)
    P = k * (k - 1) // 2
    parts, per = chunk_parts(lengths, rank, world, chunks)
    ids = np.concatenate(parts) if parts else np.zeros(0, dtype=np.int64)
    bounds = np.cumsum([0] + [len(x) for x in parts])
    chain = seqalign.ChainStream(P) if rank == 0 else None
    pen = np.zeros(max(len(ids), 1), dtype=np.int32)
    hs = np.zeros((max(len(ids), 1), 64), dtype=np.uint8)
    err = None
    pending = False
    got = 0
    try:
        try:
            eng.align_pairs_begin(ids, pxy, pgap)
            pending = True
        except Exception as e:
            err = e
        for c in range(chunks):
            rec = None
            if err is None:
                try:
                    while got < bounds[c + 1]:
                        u, p_, h_ = eng.align_pairs_poll(got)
                        if u > got:
                            pen[got:u] = p_
                            hs[got:u] = h_
                            got = u
                        elif got < bounds[c + 1]:
                            time.sleep(poll_s)
                    if on_piece is not None:
                        on_piece(c)
                    lo, hi = bounds[c], bounds[c + 1]
                    rec = pack_records(parts[c], pen[lo:hi], hs[lo:hi], per[c])
                except Exception as e:
                    err = e
            if rec is None:  # still join the collective, so no peer waits forever
                rec = pack_records([], [], [], per[c])
                rec[:, :4] = np.array([FAILED], dtype=np.int32).view(np.uint8)
            g = all_gather_records(rec, device=device, group=group)
            if err is not None:
                continue
            try:
                cid, cpen, chs = unpack_chunk(g)
            except RankFailed as e:  # every rank sees it in the same gather
                err = e
                continue
            if chain is not None:
                chain.feed(cid, cpen, chs)
        if pending:
            pending = False
            try:
                eng.align_pairs_end()
            except Exception as e:
                if err is None:
                    err = e
        if err is not None:
            raise RankFailed("rank %d: %s" % (rank, err)) from err
        if chain is None:
            return None, None, None
        return chain.finish()
    finally:
        if pending:
            try:
                eng.align_pairs_end()
            except Exception:
                pass
        if chain is not None:
            chain.close()


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
