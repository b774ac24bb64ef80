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

Communicators: RcclComm (the GPU ranks: RCCL through the library's own
nwk_comm_*, so a rank process maps one HIP runtime and one RCCL and never
imports torch) or TorchComm (torch.distributed: gloo in the CPU tests).

Streamed jobs on one node (align_sharded_streamed with a NodeRecords): an RCCL
collective cannot run while a rank's persistent fill launch holds the GPU --
the fill's 4 waves/SIMD x 128 VGPRs fill every SIMD's register file, and RCCL's
kernel needs 248-256 VGPRs and 37.7 KB of LDS per block; measured, even a
one-wave kernel waits ~8 ms until the launch drains, and reserving CUs does
not free RCCL-shaped blocks (tools/overlap_probe*.py, profiles/r05/overlap).
So the pieces' records travel to rank 0's chain through node-local shared
memory as they stream out of each rank's launch (the way sub:305-331's master
takes results as workers finish), and the records of the whole shard go
through ONE RCCL all-gather after the launch -- the collective of record, whose
result rank 0 checks against what the chain consumed.
"""
import os
import time

import numpy as np

import seqalign

REC = 72


_SHARDS = {}


def all_shards(lengths, world):
    """Every rank's LPT shard (seqalign.shard_pairs, ascending ids), computed once
    per (lengths, world): the streamed paths need all of them every step, and
    C4's eight shards cost ~20 ms of host time (inside the timed step) uncached."""
    key = (world, np.asarray(lengths, dtype=np.int64).tobytes())
    got = _SHARDS.get(key)
    if got is None:
        got = [np.sort(seqalign.shard_pairs(lengths, r, world)) for r in range(world)]
        if len(_SHARDS) > 8:
            _SHARDS.clear()
        _SHARDS[key] = got
    return got


def shard_sizes(lengths, world):
    return [len(x) for x in all_shards(lengths, world)]


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


class TorchComm:
    """torch.distributed as the communicator (gloo on CPU in the tests)."""

    def __init__(self, group=None, device=None):
        import torch.distributed as tdist

        self.dist, self.group, self.device = tdist, group, device
        self.world = tdist.get_world_size(group)
        self.rank = tdist.get_rank(group)
        self.backend = tdist.get_backend(group)

    def all_gather(self, rec):
        import torch

        t = torch.from_numpy(np.ascontiguousarray(rec))
        if self.device is not None:
            t = t.to(self.device, non_blocking=False)
        out = torch.empty((self.world * rec.shape[0],) + tuple(rec.shape[1:]), dtype=t.dtype, device=t.device)
        self.dist.all_gather_into_tensor(out, t, group=self.group)
        return out.cpu().numpy()

    def max(self, x):
        import torch

        t = torch.tensor([float(x)], dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def barrier(self):
        self.dist.barrier(group=self.group)

    def close(self):
        pass


class RcclComm:
    """RCCL through libnwk (seqalign.Comm): the GPU ranks' communicator."""

    backend = "rccl (nwk_comm)"

    def __init__(self, comm):
        self.comm = comm
        self.world, self.rank = comm.world, comm.rank

    def all_gather(self, rec):
        g = self.comm.all_gather(rec)
        return g.reshape((self.world * rec.shape[0],) + tuple(rec.shape[1:]))

    def max(self, x):
        return float(self.comm.all_reduce_max([float(x)])[0])

    def barrier(self):
        self.comm.barrier()

    def close(self):
        self.comm.close()


def process_start_time():
    """Wall-clock start of this process (s since the epoch)."""
    try:
        import psutil

        return psutil.Process().create_time()
    except Exception:
        return _IMPORT_TIME


_IMPORT_TIME = time.time()


def read_rendezvous_id(path, rank, not_before, timeout_s, poll_s=0.01, nbytes=None):
    """The RCCL unique id rank 0 wrote to `path`: only a complete file written
    after `not_before` (this rank's start) counts, so a file left by an earlier
    run that died before removing it is never used (its ncclCommInitRank would
    hang on a mismatched id)."""
    nbytes = nbytes or seqalign.COMM_ID_BYTES
    t0 = time.time()
    while True:
        try:
            if os.path.getmtime(path) >= not_before - 1.0:
                with open(path, "rb") as f:
                    uid = f.read()
                if len(uid) == nbytes:
                    return uid
        except OSError:
            pass
        if time.time() - t0 > timeout_s:
            raise RuntimeError("rank %d: no RCCL id from rank 0 at %s after %.0f s" % (rank, path, timeout_s))
        time.sleep(poll_s)


def rccl_comm(device, world, rank, timeout_s=120.0):
    """RcclComm for this rank process.  Rendezvous on the node: rank 0 writes
    the RCCL id to a file named by the launch (run_key: the launcher's run id,
    else MASTER_PORT and the ranks' common parent); the other ranks wait for a
    complete file written after they started (read_rendezvous_id).  All ranks
    of a bench run are on one node (torch.distributed.run --nnodes=1, or
    bench.py's own spawn)."""
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "nwk_rccl_id_%s" % run_key())
    if rank == 0:
        uid = seqalign.Comm.unique_id()
        tmp = path + ".tmp%d" % os.getpid()
        with open(tmp, "wb") as f:
            f.write(uid)
        os.replace(tmp, path)
    else:
        uid = read_rendezvous_id(path, rank, process_start_time(), timeout_s)
    comm = RcclComm(seqalign.Comm(device, uid, world, rank))
    comm.barrier()  # every rank has read the id
    if rank == 0:
        try:
            os.remove(path)
        except OSError:
            pass
    return comm


def default_comm(comm, device=None, group=None):
    return comm if comm is not None else TorchComm(group, device)


def all_gather_records(rec, device=None, group=None, comm=None):
    """ONE collective: every rank contributes `per` records."""
    return default_comm(comm, device, group).all_gather(rec)


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
    shards = all_shards(lengths, world)
    per = [max([len(cut(sh, c)) for sh in shards] + [1]) for c in range(chunks)]
    return [cut(shards[rank], c) for c in range(chunks)], per


def auto_chunks(P, world):
    """Pieces per rank: one.  A piece's pairs finish together at the end of its
    launch (strips: one wave per pair, one round), and a half-full launch takes
    as long as a full one, so two pieces cost a second fill: C4 at W = 8, 1
    piece 28.4 ms, 2 pieces 31.0 ms (profiles/r03/sched).
    align_sharded_pipelined keeps the piece machinery for chunks > 1."""
    return 1


def failed_block(per):
    """A padded record block with every record tagged FAILED."""
    rec = pack_records([], [], [], per)
    rec[:, :4] = np.array([FAILED], dtype=np.int32).view(np.uint8)
    return rec


class PipelinedShard:
    """Rank side of align_sharded_pipelined: the shard in pieces of ascending
    canonical ids, piece c+1 aligning (Engine.align_pairs_begin) while piece
    c's block is exchanged.  block(c) returns piece c's padded record block --
    FAILED-tagged once this rank has failed, so it still joins every
    collective.  The tests and tools/shardtime.py drive the same object per
    rank on one GPU and stand in for the all-gather with a concatenation."""

    def __init__(self, eng, parts, per, pxy, pgap, on_piece=None):
        self.eng, self.parts, self.per, self.pxy, self.pgap = eng, parts, per, pxy, pgap
        self.on_piece = on_piece
        self.err = None       # this rank's own failure
        self.pending = False  # an align_pairs_begin not yet ended

    def start(self):
        try:
            self.eng.align_pairs_begin(self.parts[0], self.pxy, self.pgap)
            self.pending = True
        except Exception as e:
            self.err = e

    def block(self, c):
        if self.err is None:
            try:
                self.pending = False
                pen, hs = self.eng.align_pairs_end()
                if self.on_piece is not None:
                    self.on_piece(c)
                if c + 1 < len(self.parts):
                    self.eng.align_pairs_begin(self.parts[c + 1], self.pxy, self.pgap)
                    self.pending = True
                return pack_records(self.parts[c], pen, hs, self.per[c])
            except Exception as e:
                self.err = e
        return failed_block(self.per[c])

    def finish(self):
        """Ends a call still in flight (a peer failed first); returns this rank's error."""
        if self.pending:
            self.pending = False
            try:
                self.eng.align_pairs_end()
            except Exception:
                pass
        return self.err


class StreamedShard:
    """Rank side of align_sharded_streamed: the whole shard as ONE launch over
    its ids in ascending canonical order (the engine built with
    finalize="fused"), its per-pair records polled as they stream out of the
    fill launch (Engine.align_pairs_poll).  block(c) waits until every record
    of piece c is in and returns its padded block (FAILED-tagged once this
    rank has failed).  finish() ends the launch: errors that only the end of
    the call reports (the device error word, a fused record that fails its
    checks) surface there, after every piece's exchange -- hence the final
    status collective in align_sharded_streamed."""

    def __init__(self, eng, parts, per, pxy, pgap, poll_s=50e-6, on_piece=None):
        self.eng, self.parts, self.per, self.pxy, self.pgap = eng, parts, per, pxy, pgap
        self.poll_s, self.on_piece = poll_s, on_piece
        self.ids = np.concatenate(parts) if parts else np.zeros(0, dtype=np.int64)
        self.bounds = np.cumsum([0] + [len(x) for x in parts])
        n = max(len(self.ids), 1)
        self.pen = np.zeros(n, dtype=np.int32)
        self.hs = np.zeros((n, 64), dtype=np.uint8)
        self.got = 0
        self.err = None
        self.pending = False

    def start(self):
        try:
            self.eng.align_pairs_begin(self.ids, self.pxy, self.pgap)
            self.pending = True
        except Exception as e:
            self.err = e

    def block(self, c):
        import time

        if self.err is None:
            try:
                hi = self.bounds[c + 1]
                while self.got < hi:
                    u, p_, h_ = self.eng.align_pairs_poll(self.got)
                    if u > self.got:
                        self.pen[self.got:u] = p_
                        self.hs[self.got:u] = h_
                        self.got = u
                    elif self.got < hi:
                        time.sleep(self.poll_s)
                if self.on_piece is not None:
                    self.on_piece(c)
                lo = self.bounds[c]
                return pack_records(self.parts[c], self.pen[lo:hi], self.hs[lo:hi], self.per[c])
            except Exception as e:
                self.err = e
        return failed_block(self.per[c])

    def finish(self):
        """Ends the launch; returns this rank's error (None on success)."""
        if self.pending:
            self.pending = False
            try:
                self.eng.align_pairs_end()
            except Exception as e:
                if self.err is None:
                    self.err = e
        return self.err


class _NodeSegment:
    """A POSIX shared-memory segment of one node's ranks, named by the run key:
    rank 0 creates it (a stale one of the same name is replaced) and stamps it
    with a nonce that every rank receives through the communicator before
    attaching, so no rank can read a segment left by an earlier run.
    layout(world) -> (header bytes after the nonce line, data bytes)."""

    def _open(self, comm, hdr_b, data_b, key=None):
        from multiprocessing import shared_memory

        self.world, self.rank = comm.world, comm.rank
        key = key or run_key()
        self.name = "%s_%s" % (self.PREFIX, key)
        self.data_off = 64 + (hdr_b + 63) // 64 * 64
        size = self.data_off + max(int(data_b), 1)
        nonce = 0
        if self.rank == 0:
            try:  # a segment left by a run that died
                old = shared_memory.SharedMemory(name=self.name)
                old.close()
                old.unlink()
            except FileNotFoundError:
                pass
            self.shm = shared_memory.SharedMemory(name=self.name, create=True, size=size)
            # flags cleared BEFORE the nonce goes out: a peer may publish as soon
            # as it has it (clearing after the collective erased a fast peer's
            # first flag, and rank 0 waited for it forever)
            np.ndarray((hdr_b // 8,), dtype=np.int64, buffer=self.shm.buf, offset=64)[:] = 0
            nonce = int.from_bytes(os.urandom(6), "little") | 1
            np.ndarray((1,), dtype=np.int64, buffer=self.shm.buf)[0] = nonce
        nonce = int(comm.max(float(nonce)))  # rank 0's nonce (< 2^53), after it created the segment
        if self.rank != 0:
            self.shm = shared_memory.SharedMemory(name=self.name)
            # Python < 3.13 registers an attached segment with this process's
            # resource tracker, which would unlink it (and warn) when a peer
            # exits: only rank 0 owns the segment's lifetime
            try:
                from multiprocessing import resource_tracker
                resource_tracker.unregister(self.shm._name, "shared_memory")
            except Exception:
                pass
            if int(np.ndarray((1,), dtype=np.int64, buffer=self.shm.buf)[0]) != nonce:
                raise RuntimeError("rank %d: node record segment %s is not this run's" % (self.rank, self.name))

    def close(self):
        shm, self.shm = getattr(self, "shm", None), None
        if shm is None:
            return
        self._drop_views()
        shm.close()
        if self.rank == 0:
            try:
                # (ranks spawned by one parent share its resource tracker, where a
                # peer's unregister above removed the name: re-register it so the
                # unregister inside unlink() finds it)
                from multiprocessing import resource_tracker
                resource_tracker.register(shm._name, "shared_memory")
            except Exception:
                pass
            try:
                shm.unlink()
            except FileNotFoundError:
                pass


class NodeRecords(_NodeSegment):
    """Per-piece record blocks of every rank of one node, in POSIX shared
    memory: rank r's block of piece c (per[c] records) at slot (r, c), then its
    flag (int64) set to the step's token.  Stores are ordered by the x86-64
    memory model (TSO, every MI355X host): a reader that sees the flag sees the
    block.  Segment lifetime and nonce: _NodeSegment."""

    PREFIX = "nwk_rec"

    def __init__(self, comm, chunks, per, key=None):
        self.chunks = chunks
        self.per = [int(x) for x in per]
        self.pre = np.cumsum([0] + self.per)
        self.sum_per = int(self.pre[-1])
        self._open(comm, 8 * comm.world * chunks, comm.world * self.sum_per * REC, key)
        self.flags = np.ndarray((self.world, chunks), dtype=np.int64, buffer=self.shm.buf, offset=64)
        self.data = np.ndarray((self.world, self.sum_per, REC), dtype=np.uint8, buffer=self.shm.buf,
                               offset=self.data_off)

    def _drop_views(self):
        self.flags = self.data = None

    def publish(self, c, block, token):
        """This rank's padded block of piece c, then its flag."""
        self.data[self.rank, self.pre[c]:self.pre[c + 1]] = block
        self.flags[self.rank, c] = token

    def wait(self, c, token, poll_s=20e-6, timeout_s=600.0):
        """Every rank's block of piece c (rank-major, as an all-gather returns them)."""
        t0 = time.time()
        while not (self.flags[:, c] == token).all():
            if time.time() - t0 > timeout_s:
                raise RuntimeError("node records: piece %d not published by every rank in %.0f s" % (c, timeout_s))
            time.sleep(poll_s)
        return self.data[:, self.pre[c]:self.pre[c + 1]].reshape(-1, REC).copy()

    def shard_blocks(self):
        """Every rank's whole padded shard (rank-major), as it is in the segment NOW
        (a peer that has returned may already publish its next call's pieces)."""
        return self.data.reshape(-1, REC)

    def as_shards(self, taken):
        """The pieces wait() returned, in piece order, rearranged rank-major over
        whole shards -- the layout of the all-gather of every rank's shard."""
        return np.concatenate([t.reshape(self.world, -1, REC) for t in taken], axis=1).reshape(-1, REC)


class NodeStream(_NodeSegment):
    """Per-record exchange of one node's streamed ranks (round 6): rank r's
    shard records at slots (r, 0 .. n_r) in its shard order (ascending
    canonical ids), and one progress word per rank, on its own cache line:
    token << 32 | records published so far (FAILED_COUNT: the rank failed),
    stored after the records (x86-TSO: a reader that sees the count sees the
    records).  Rank 0's chain takes each record as soon as its rank has
    published it -- the master of sub:305-331 takes each worker's result as it
    arrives -- instead of a piece of 1/16 of the canonical ids at a time."""

    PREFIX = "nwk_str"
    FAILED_COUNT = 0xFFFFFFFF

    def __init__(self, comm, per, key=None):
        self.per = max(int(per), 1)
        self._open(comm, 64 * comm.world, comm.world * self.per * REC, key)
        self.words = np.ndarray((self.world, 8), dtype=np.int64, buffer=self.shm.buf, offset=64)
        self.data = np.ndarray((self.world, self.per, REC), dtype=np.uint8, buffer=self.shm.buf,
                               offset=self.data_off)

    def _drop_views(self):
        self.words = self.data = None

    def publish(self, lo, hi, block, token):
        """This rank's records lo .. hi (its shard order), then its progress word."""
        self.data[self.rank, lo:hi] = block
        self.words[self.rank, 0] = (int(token) << 32) | int(hi)

    def fail(self, token):
        self.words[self.rank, 0] = (int(token) << 32) | self.FAILED_COUNT

    def progress(self, token):
        """Per rank: records published in this call (-1: none yet), FAILED_COUNT: failed."""
        w = self.words[:, 0].copy()
        return np.where((w >> 32) == int(token), w & 0xFFFFFFFF, -1)

    def take(self, r, lo, hi):
        return self.data[r, lo:hi].copy()


def run_key():
    """A name shared by the ranks of one launch: the launcher's run id
    (TORCHELASTIC_RUN_ID; NWK_RUN_ID from bench.py's own spawn), else
    MASTER_PORT and the ranks' common parent process."""
    rid = os.environ.get("NWK_RUN_ID") or os.environ.get("TORCHELASTIC_RUN_ID")
    if rid:
        return "".join(ch for ch in rid if ch.isalnum())[:40] + "_%s" % os.environ.get("MASTER_PORT", "0")
    return "%s_%s" % (os.environ.get("MASTER_PORT", "0"), os.getppid())


def node_local(world):
    """All ranks of the job on this node (torchrun's LOCAL_WORLD_SIZE, or bench.py's own spawn)."""
    return int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) == world


def any_rank_failed(failed, comm):
    """One status collective (all-reduce MAX of a flag): True on every rank
    when any rank failed."""
    return comm.max(1.0 if failed else 0.0) > 0.0


def _exchange(shard, chunks, rank, P, comm, final_status):
    """The collective side shared by both pipelines: one all-gather per piece,
    rank 0's chain worker fed per piece as it arrives (sub:305-331 collects
    results as they arrive, sub:334-337 chains)."""
    chain = seqalign.ChainStream(P) if rank == 0 else None
    err = None  # a peer's failure seen in a gather
    try:
        shard.start()
        for c in range(chunks):
            g = comm.all_gather(shard.block(c))
            if err is not None or shard.err is not None:
                continue
            try:
                cid, cpen, chs = unpack_chunk(g)
            except RankFailed as e:  # every rank sees it in the same gather
                err = e
                continue
            if chain is not None:
                chain.feed(cid, cpen, chs)
        own = shard.finish()
        err = own if own is not None else err
        if final_status and any_rank_failed(err is not None, comm) and err is None:
            err = RankFailed("a peer rank failed after the last piece was exchanged")
        if err is not None:
            raise RankFailed("rank %d: %s" % (rank, err)) from err
        if chain is None:
            return None, None, None
        return chain.finish()
    finally:
        shard.finish()
        if chain is not None:
            chain.close()


def align_sharded_pipelined(eng, lengths, pxy, pgap, rank, world, chunks=1, device=None, group=None,
                            on_piece=None, comm=None):
    """The shard in `chunks` pieces of ascending canonical ids: piece c+1 aligns
    on the GPU (Engine.align_pairs_begin) while piece c's records go through
    their all-gather and rank 0's chain worker (seqalign.ChainStream) advances
    over them -- sub:305-337 collects results as they arrive and then chains;
    here the chain of all but the last piece hides behind the alignment.
    Returns (hash, penalties[P], hashes[P,64]) on rank 0, (None, None, None)
    elsewhere.  Same failure contract as align_sharded: a failing rank joins
    every remaining collective with FAILED records, and every rank raises
    (each piece's end() runs before its gather, so no final status is needed)."""
    k = len(lengths)
    P = k * (k - 1) // 2
    parts, per = chunk_parts(lengths, rank, world, chunks)
    shard = PipelinedShard(eng, parts, per, pxy, pgap, on_piece=on_piece)
    return _exchange(shard, chunks, rank, P, default_comm(comm, device, group), final_status=False)


def _exchange_node(shard, chunks, rank, P, comm, node, token):
    """The streamed pipeline with node-local piece exchange (NodeRecords):
    every rank publishes each piece's block as its records are in, rank 0's
    chain worker takes piece c once every rank has published it, and after the
    launch the whole shard's records go through ONE all-gather (RCCL on the GPU
    ranks) -- rank 0 checks that it returns exactly what the chain consumed.
    Failure contract as _exchange: a failed rank publishes FAILED-tagged blocks
    and joins both collectives; every rank raises."""
    chain = seqalign.ChainStream(P) if rank == 0 else None
    err = None
    blocks = []
    taken = []  # rank 0: the pieces the chain took (copies: peers reuse the segment once they return)
    try:
        shard.start()
        for c in range(chunks):
            b = shard.block(c)
            blocks.append(b)
            node.publish(c, b, token)
            if chain is None or err is not None:
                continue
            got = node.wait(c, token)
            taken.append(got)
            try:
                cid, cpen, chs = unpack_chunk(got)
            except RankFailed as e:
                err = e
                continue
            chain.feed(cid, cpen, chs)
        own = shard.finish()
        err = own if own is not None else err
        mine = np.concatenate(blocks) if own is None else failed_block(node.sum_per)
        g = comm.all_gather(mine)  # the collective of record: every rank's whole shard
        if any_rank_failed(err is not None, comm) and err is None:
            err = RankFailed("a peer rank failed")
        if err is not None:
            raise RankFailed("rank %d: %s" % (rank, err)) from err
        if chain is None:
            return None, None, None
        # (against the copies taken: after the last collective a peer may already
        # publish its next call's pieces into the live segment)
        if not np.array_equal(np.asarray(g, dtype=np.uint8).reshape(-1, REC), node.as_shards(taken)):
            raise RuntimeError("rank 0: the all-gathered records differ from the node records the chain took")
        return chain.finish()
    finally:
        shard.finish()
        if chain is not None:
            chain.close()


def align_sharded_streamed(eng, lengths, pxy, pgap, rank, world, chunks=8, device=None, group=None,
                           on_piece=None, poll_s=50e-6, comm=None, node=None, token=1):
    """The shard as ONE launch whose per-pair records stream to the host as
    pairs are hashed inside the fill launch (StreamedShard).  Piece c -- the
    shard's ids below the global threshold P (c+1) / chunks -- goes through its
    all-gather as soon as all of its records are in, and rank 0's chain worker
    advances over it while the rest of the shard still aligns.
    Same return value and failure contract as align_sharded_pipelined, plus one
    status collective after the launch has ended: a rank whose failure only the
    end of its call reports (after its records were already exchanged) makes
    every rank, rank 0 included, raise instead of returning a hash.
    node (a NodeRecords over the same chunks, all ranks on this node): the
    pieces reach rank 0 through shared memory and ONE all-gather follows the
    launch (_exchange_node); token: this call's flag value (the same on every
    rank, different from the previous call's)."""
    k = len(lengths)
    P = k * (k - 1) // 2
    parts, per = chunk_parts(lengths, rank, world, chunks)
    shard = StreamedShard(eng, parts, per, pxy, pgap, poll_s=poll_s, on_piece=on_piece)
    if node is not None:
        return _exchange_node(shard, chunks, rank, P, default_comm(comm, device, group), node, token)
    return _exchange(shard, chunks, rank, P, default_comm(comm, device, group), final_status=True)


def stream_per(lengths, world):
    """The padded shard size of the per-record exchange (the largest shard)."""
    return max(shard_sizes(lengths, world) + [1])


def align_sharded_records(eng, lengths, pxy, pgap, rank, world, node, token, comm=None, device=None, group=None,
                          poll_s=20e-6, timeout_s=600.0, on_first=None):
    """The streamed shard (ONE launch per rank, the fused device finalize) with
    every record handed to rank 0's chain as soon as it is out: each rank polls
    its launch (Engine.align_pairs_poll) and publishes the new records into the
    node segment (NodeStream); rank 0 feeds every record any rank has published
    to its chain worker, which advances over the canonical prefix as it
    completes (skel:159).  For uniform lengths the LPT shard is round-robin over
    canonical ids and every rank aligns its ids in ascending order, so the
    prefix grows from the first records of all ranks at once.
    After the launches: ONE all-gather of the padded shards (the collective of
    record, RCCL on the GPU ranks) that rank 0 checks against the records its
    chain took, and one status collective.  Failure contract as
    align_sharded_streamed: a failed rank marks its progress word, joins both
    collectives with FAILED records, and every rank raises.
    on_first(): called on rank 0 when its chain has taken the first record.
    Returns (hash, penalties[P], hashes[P,64]) on rank 0, (None, None, None) elsewhere."""
    comm = default_comm(comm, device, group)
    k = len(lengths)
    P = k * (k - 1) // 2
    sizes = shard_sizes(lengths, world)
    per = node.per
    ids = all_shards(lengths, world)[rank]
    n = len(ids)
    mine = pack_records([], [], [], per)
    chain = seqalign.ChainStream(P) if rank == 0 else None
    taken = np.stack([pack_records([], [], [], per) for _ in range(world)]) if rank == 0 else None
    seen = [0] * world
    own_err = None
    err = None  # a failure rank 0 saw in a progress word
    pending = False
    got = 0
    first = True
    try:
        try:
            eng.align_pairs_begin(ids, pxy, pgap)
            pending = True
        except Exception as e:
            own_err = e
            node.fail(token)
        t0 = time.time()
        while True:
            moved = False
            if own_err is None and got < n:
                try:
                    u, p_, h_ = eng.align_pairs_poll(got)
                    if u > got:
                        blk = pack_records(ids[got:u], p_, h_, u - got)
                        mine[got:u] = blk
                        node.publish(got, u, blk, token)
                        got = u
                        moved = True
                except Exception as e:
                    own_err = e
                    node.fail(token)
            own_done = own_err is not None or got >= n
            if chain is not None and err is None:
                cnt = node.progress(token)
                for r in range(world):
                    c = int(cnt[r])
                    if c == NodeStream.FAILED_COUNT:
                        err = RankFailed("rank %d failed while streaming its records" % r)
                        break
                    if c > seen[r]:
                        blk = node.take(r, seen[r], c)
                        taken[r, seen[r]:c] = blk
                        cid, cpen, chs = unpack_chunk(blk)
                        chain.feed(cid, cpen, chs)
                        if first and on_first is not None:
                            on_first()
                        first = False
                        seen[r] = c
                        moved = True
            if own_done and (chain is None or err is not None or all(seen[r] >= sizes[r] for r in range(world))):
                break
            if not moved:
                if time.time() - t0 > timeout_s:
                    raise RuntimeError("node stream: records not published by every rank in %.0f s" % timeout_s)
                time.sleep(poll_s)
        if pending:
            pending = False
            try:
                eng.align_pairs_end()
            except Exception as e:
                if own_err is None:
                    own_err = e
        g = comm.all_gather(mine if own_err is None else failed_block(per))  # the collective of record
        err = own_err if own_err is not None else err
        if any_rank_failed(err is not None, comm) and err is None:
            err = RankFailed("a peer rank failed")
        if err is not None:
            raise RankFailed("rank %d: %s" % (rank, err)) from err
        if chain is None:
            return None, None, None
        if not np.array_equal(np.asarray(g, dtype=np.uint8).reshape(-1, REC), taken.reshape(-1, REC)):
            raise RuntimeError("rank 0: the all-gathered records differ from the node records the chain took")
        return chain.finish()
    finally:
        if pending:
            try:
                eng.align_pairs_end()
            except Exception:
                pass
        if chain is not None:
            chain.close()


def emulate_ranks(make_shard, world, chunks, P):
    """Runs every rank's shard one after another in this process (one GPU
    standing in for W) and exchanges the blocks by concatenation in rank
    order -- exactly what all_gather_into_tensor returns -- then chains.
    make_shard(rank) -> a started-able PipelinedShard / StreamedShard.
    Returns (hash, penalties[P], hashes[P,64], per-rank per-piece ready times in s)."""
    import time

    blocks = [[None] * chunks for _ in range(world)]
    ready = np.zeros((world, chunks))
    for r in range(world):
        sh = make_shard(r)
        t0 = time.perf_counter()
        sh.start()
        for c in range(chunks):
            blocks[r][c] = sh.block(c)
            ready[r, c] = time.perf_counter() - t0
        err = sh.finish()
        if err is not None:
            raise RankFailed("rank %d: %s" % (r, err)) from err
    chain = seqalign.ChainStream(P)
    try:
        for c in range(chunks):
            cid, cpen, chs = unpack_chunk(np.concatenate([blocks[r][c] for r in range(world)]))
            chain.feed(cid, cpen, chs)
        h, pen, hs = chain.finish()
    finally:
        chain.close()
    return h, pen, hs, ready


def align_sharded(align_fn, lengths, pxy, pgap, rank, world, device=None, group=None, comm=None):
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
        rec = failed_block(per)
    g = all_gather_records(rec, device=device, group=group, comm=comm)
    if err is not None:
        raise RankFailed("rank %d: %s" % (rank, err)) from err
    pen_all, hs_all = unpack_records(g, P)
    return pen_all, hs_all, ids
