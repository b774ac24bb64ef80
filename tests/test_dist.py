"""world_size-2 gloo run of the multi-GPU layer on CPU.

The shard -> records -> ONE all_gather -> canonical reassembly -> chain path
of dist.py runs exactly as on the GPUs; only the per-rank aligner is swapped
for the CPU oracle (test infrastructure), since this container has no GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ORACLE, PKG, case_input, load_golden

CASES = [c for c in load_golden() if c["name"] in ("mseq1", "xulin_test", "ragged", "k2_same", "k3_T_GGGG")]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cases, q):
    import sys

    for p in (PKG, ORACLE):
        sys.path.insert(0, p)
    import numpy as np

    import dist as nwdist
    import oracle
    import seqalign

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for name, pxy, pgap, genes in cases:
            def align_fn(ids, pxy_, pgap_):
                pen, hs = [], []
                for p in ids:
                    i, j = seqalign.pair_ij(int(p))
                    pe, a1, a2 = oracle.pair(genes[i], genes[j], pxy_, pgap_)
                    pen.append(pe)
                    hs.append(list(bytes.fromhex(oracle.problem_hash(a1, a2))))
                return np.array(pen, dtype=np.int32), np.array(hs, dtype=np.uint8).reshape(-1, 64)

            lengths = [len(g) for g in genes]
            pen, hs, ids = nwdist.align_sharded(align_fn, lengths, pxy, pgap, rank, world)
            h = seqalign.chain_hash(hs)
            q.put((rank, name, h, [int(v) for v in pen], len(ids)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_gather_matches_golden(world):
    cases = []
    for c in CASES:
        pxy, pgap, genes = case_input(c)
        cases.append((c["name"], pxy, pgap, genes))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world * len(cases))]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gold = {c["name"]: c for c in CASES}
    per_case = {}
    for rank, name, h, pen, n in out:
        assert h == gold[name]["hash"], (rank, name)
        assert pen == gold[name]["penalties"]
        per_case.setdefault(name, 0)
        per_case[name] += n
    for c in CASES:
        k = len(case_input(c)[2])
        assert per_case[c["name"]] == k * (k - 1) // 2


def _failing_worker(rank, world, port, genes, q):
    import sys

    for p in (PKG, ORACLE):
        sys.path.insert(0, p)
    import numpy as np

    import dist as nwdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def align_fn(ids, pxy, pgap):
            if rank == 1:
                raise RuntimeError("injected NWK_EKERNEL on rank 1")
            return np.zeros(len(ids), dtype=np.int32), np.zeros((len(ids), 64), dtype=np.uint8)

        try:
            nwdist.align_sharded(align_fn, [len(g) for g in genes], 3, 2, rank, world)
            q.put((rank, "returned"))
        except nwdist.RankFailed as e:
            q.put((rank, "raised: %s" % e))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_failing_rank_raises_everywhere(world):
    """One rank's aligner raises: it still joins the ONE all-gather with
    records tagged FAILED, and every rank raises RankFailed (none hangs)."""
    genes = [b"ACGT" * 5, b"AC" * 7, b"GATTACA", b"T" * 11, b"CAT" * 4]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_failing_worker, args=(r, world, port, genes, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(out) == list(range(world))
    for r, msg in out.items():
        assert msg.startswith("raised:"), (r, msg)
    assert "injected" in out[1]


class _OracleEngine:
    """Test stand-in for seqalign.Engine's begin/end pair (the CPU oracle as
    the per-rank aligner -- test infrastructure; there is no GPU here).
    fail_at: raise in the end() of that piece."""

    def __init__(self, genes, fail_at=None):
        self.genes, self.fail_at, self.calls, self.ids = genes, fail_at, 0, None

    def align_pairs_begin(self, ids, pxy, pgap):
        assert self.ids is None, "one piece in flight"
        self.ids, self.pxy, self.pgap = list(ids), pxy, pgap

    def align_pairs_end(self):
        import numpy as np

        import oracle
        import seqalign

        ids, self.ids = self.ids, None
        self.calls += 1
        if self.fail_at is not None and self.calls - 1 == self.fail_at:
            raise RuntimeError("injected NWK_EKERNEL in piece %d" % self.fail_at)
        pen, hs = [], []
        for p in ids:
            i, j = seqalign.pair_ij(int(p))
            pe, a1, a2 = oracle.pair(self.genes[i], self.genes[j], self.pxy, self.pgap)
            pen.append(pe)
            hs.append(list(bytes.fromhex(oracle.problem_hash(a1, a2))))
        return np.array(pen, dtype=np.int32), np.array(hs, dtype=np.uint8).reshape(-1, 64)


def _pipelined_worker(rank, world, port, cases, chunks, fail, q):
    import sys

    for p in (PKG, ORACLE):
        sys.path.insert(0, p)
    import dist as nwdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for name, pxy, pgap, genes in cases:
            eng = _OracleEngine(genes, fail_at=1 if (fail and rank == 1) else None)
            try:
                h, pen, _ = nwdist.align_sharded_pipelined(eng, [len(g) for g in genes], pxy, pgap, rank, world,
                                                           chunks=chunks)
                q.put((rank, name, h, None if pen is None else [int(v) for v in pen]))
            except nwdist.RankFailed as e:
                q.put((rank, name, "raised: %s" % e, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,chunks", [(2, 1), (2, 3), (3, 2), (3, 5)])
def test_gloo_pipelined_chunks_match_golden(world, chunks):
    """dist.align_sharded_pipelined: each rank's shard in pieces of ascending
    canonical ids, one all-gather per piece while the next piece aligns, rank
    0's streaming chain (nwk_chain_*) fed per piece -- the answer hash and
    penalties of the reference (golden) for any number of pieces."""
    cases = []
    for c in CASES:
        pxy, pgap, genes = case_input(c)
        cases.append((c["name"], pxy, pgap, genes))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipelined_worker, args=(r, world, port, cases, chunks, False, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world * len(cases))]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gold = {c["name"]: c for c in CASES}
    for rank, name, h, pen in out:
        if rank == 0:
            assert h == gold[name]["hash"], name
            assert pen == gold[name]["penalties"], name
        else:
            assert h is None


def test_gloo_pipelined_failing_piece_raises_everywhere():
    """Rank 1's second piece fails while its third is pending: it joins every
    remaining all-gather with FAILED records and all ranks raise (none hangs)."""
    genes = [b"ACGT" * 5, b"AC" * 7, b"GATTACA", b"T" * 11, b"CAT" * 4, b"GG" * 6, b"TACG" * 3]
    cases = [("f", 3, 2, genes)]
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipelined_worker, args=(r, world, port, cases, 4, True, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {r: h for r, _, h, _ in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, msg in out.items():
        assert isinstance(msg, str) and msg.startswith("raised:"), (r, msg)
    assert "injected" in out[1]


class _OracleStreamEngine(_OracleEngine):
    """The streamed engine's begin / poll / end over the CPU oracle: poll
    returns the records in order, a few pairs per call (test infrastructure).
    fail_end: end() raises after every record has been polled -- the device
    error word that only align_pairs_end reports."""

    def __init__(self, genes, fail_end=False, fail_poll=False):
        super().__init__(genes)
        self.fail_end = fail_end
        self.fail_poll = fail_poll  # poll raises once some records are out (a device error mid-launch)

    def align_pairs_begin(self, ids, pxy, pgap):
        super().align_pairs_begin(ids, pxy, pgap)
        self._pen, self._hs = _OracleEngine.align_pairs_end(self)  # computed up front, released by poll
        self.ids, self._n = list(ids), 0

    def align_pairs_poll(self, start=0):
        if self.fail_poll and start > 0:
            raise RuntimeError("injected NWK_EKERNEL while polling")
        self._n = min(len(self.ids), self._n + 3)
        return self._n, self._pen[start:self._n].copy(), self._hs[start:self._n].copy()

    def align_pairs_end(self):
        self.ids = None
        if self.fail_end:
            raise RuntimeError("injected NWK_EKERNEL at align_pairs_end")
        return self._pen, self._hs


def _streamed_worker(rank, world, port, cases, chunks, fail, q, node_records=False, steps=1, scorings=None):
    import sys

    for p in (PKG, ORACLE):
        sys.path.insert(0, p)
    import dist as nwdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for name, pxy, pgap, genes in cases:
            lens = [len(g) for g in genes]
            node = None
            if node_records == "records":  # every record through node shared memory (NodeStream)
                node = nwdist.NodeStream(nwdist.TorchComm(), nwdist.stream_per(lens, world))
            elif node_records:  # pieces through node shared memory, then ONE all-gather
                node = nwdist.NodeRecords(nwdist.TorchComm(), chunks, nwdist.chunk_parts(lens, rank, world, chunks)[1])
            try:
                for step in range(1, steps + 1):  # (the segment is reused across steps: token = step)
                    eng = _OracleStreamEngine(genes, fail_end=fail is True and rank == world - 1,
                                              fail_poll=fail == "poll" and rank == world - 1)
                    sp, sg = scorings[step - 1] if scorings else (pxy, pgap)
                    try:
                        if node_records == "records":
                            h, pen, _ = nwdist.align_sharded_records(eng, lens, sp, sg, rank, world, node, step,
                                                                     poll_s=0.0, timeout_s=120.0)
                        else:
                            h, pen, _ = nwdist.align_sharded_streamed(eng, lens, sp, sg, rank, world, chunks=chunks,
                                                                      poll_s=0.0, node=node, token=step)
                        q.put((rank, "%s@%d,%d" % (name, sp, sg) if scorings else name, h,
                               None if pen is None else [int(v) for v in pen]))
                    except nwdist.RankFailed as e:
                        q.put((rank, name, "raised: %s" % e, None))
            finally:
                if node is not None:
                    node.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,chunks,node", [(2, 1, False), (3, 4, False), (2, 1, True), (3, 4, True),
                                               (2, 1, "records"), (3, 1, "records")])
def test_gloo_streamed_pieces_match_golden(world, chunks, node):
    """dist.align_sharded_streamed (one launch per rank, records polled as they
    stream; one all-gather per piece, or -- node=True -- the pieces through
    node shared memory (NodeRecords) and one all-gather of the whole shards,
    checked against what the chain took; final status collective): the answer
    hash and penalties of the reference (golden) on rank 0, over two steps that
    reuse the node segment."""
    cases = []
    for c in CASES:
        pxy, pgap, genes = case_input(c)
        cases.append((c["name"], pxy, pgap, genes))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    steps = 2 if node else 1
    procs = [ctx.Process(target=_streamed_worker, args=(r, world, port, cases, chunks, False, q, node, steps))
             for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world * len(cases) * steps)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gold = {c["name"]: c for c in CASES}
    for rank, name, h, pen in out:
        if rank == 0:
            assert h == gold[name]["hash"], name
            assert pen == gold[name]["penalties"], name
        else:
            assert h is None


@pytest.mark.parametrize("world,mode", [(2, True), (3, True), (3, "records")])
def test_gloo_node_records_consecutive_calls_different_scorings(world, mode):
    """consecutive streamed calls with DIFFERENT records on one
    NodeRecords segment.  A peer that has returned publishes its next call's
    pieces into the live segment while rank 0 may still be checking the last
    all-gather -- rank 0 compares against the copies its chain took, so every
    call's hash equals the oracle's for its own scoring."""
    import oracle

    c = CASES[0]
    _, _, genes = case_input(c)
    scorings = [(3, 2), (5, 1), (1, 1), (3, 2)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    cases = [(c["name"], 0, 0, genes)]
    procs = [ctx.Process(target=_streamed_worker, args=(r, world, port, cases, 3, False, q, mode, len(scorings),
                                                       scorings)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world * len(scorings))]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = {}
    for sp, sg in scorings:
        h, pen, _ = oracle.all_pairs(genes, sp, sg)
        want["%s@%d,%d" % (c["name"], sp, sg)] = (h, pen)
    for rank, name, h, pen in out:
        if rank == 0:
            assert (h, pen) == want[name], name
        else:
            assert h is None


@pytest.mark.parametrize("world,node,fail", [(2, False, True), (3, False, True), (2, True, True), (3, True, True),
                                             (2, "records", True), (3, "records", True), (3, "records", "poll")])
def test_gloo_streamed_failure_at_end_raises_everywhere(world, node, fail):
    """The last rank's error surfaces only at align_pairs_end, after all of its
    records were exchanged and chained by rank 0: the final status collective
    makes every rank -- rank 0 included -- raise instead of returning a hash
    (also when the pieces went through node shared memory)."""
    genes = [b"ACGT" * 5, b"AC" * 7, b"GATTACA", b"T" * 11, b"CAT" * 4, b"GG" * 6, b"TACG" * 3]
    cases = [("f", 3, 2, genes)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_streamed_worker, args=(r, world, port, cases, 3, fail, q, node))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {r: h for r, _, h, _ in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, msg in out.items():
        assert isinstance(msg, str) and msg.startswith("raised:"), (r, msg)
    assert "injected" in out[world - 1]


def test_emulated_ranks_match_golden():
    """dist.emulate_ranks (the one-GPU stand-in for W ranks that the full-size
    GPU tests and tools/shardtime.py use): the same rank-side objects, the
    all-gather replaced by concatenation in rank order."""
    import sys

    for p in (PKG, ORACLE):
        if p not in sys.path:
            sys.path.insert(0, p)
    import dist as nwdist

    for c in CASES:
        pxy, pgap, genes = case_input(c)
        lengths = [len(g) for g in genes]
        P = len(genes) * (len(genes) - 1) // 2
        for world, chunks, streamed in ((2, 1, False), (3, 2, True), (4, 3, False)):
            def make(r):
                parts, per = nwdist.chunk_parts(lengths, r, world, chunks)
                if streamed:
                    return nwdist.StreamedShard(_OracleStreamEngine(genes), parts, per, pxy, pgap, poll_s=0.0)
                return nwdist.PipelinedShard(_OracleEngine(genes), parts, per, pxy, pgap)

            h, pen, _, ready = nwdist.emulate_ranks(make, world, chunks, P)
            assert h == c["hash"], (c["name"], world, chunks)
            assert [int(v) for v in pen] == c["penalties"]
            assert ready.shape == (world, chunks)


class _FakeComm:
    """seqalign.Comm stand-in for the RCCL rendezvous (no device, no RCCL)."""

    made = []

    def __init__(self, device, uid, world, rank):
        self.uid, self.world, self.rank = uid, world, rank
        _FakeComm.made.append(self)

    @staticmethod
    def unique_id():
        return bytes(range(128))

    def barrier(self):
        pass

    def close(self):
        pass


def test_rccl_rendezvous_stale_file_timeout_and_length(tmp_path, monkeypatch):
    """dist.rccl_comm's id rendezvous with a fake communicator: a file left by
    an earlier run (older than this rank's start) is never used, a short file
    is waited past, a missing id times out, and rank 0's fresh id is taken."""
    import sys
    import time

    sys.path.insert(0, PKG)
    import dist as nwdist
    import seqalign

    monkeypatch.setenv("TMPDIR", str(tmp_path))
    monkeypatch.setenv("NWK_RUN_ID", "rdvtest")
    monkeypatch.setenv("MASTER_PORT", "4242")
    monkeypatch.setattr(seqalign, "Comm", _FakeComm)
    path = tmp_path / ("nwk_rccl_id_%s" % nwdist.run_key())
    # a stale id from a run that died: ignored, so rank 1 times out
    path.write_bytes(b"\x07" * 128)
    old = time.time() - 3600
    os.utime(path, (old, old))
    with pytest.raises(RuntimeError, match="no RCCL id"):
        nwdist.rccl_comm(0, 2, 1, timeout_s=0.3)
    # a fresh but short file (rank 0 mid-write): waited past, then timeout
    path.write_bytes(b"\x07" * 100)
    with pytest.raises(RuntimeError, match="no RCCL id"):
        nwdist.rccl_comm(0, 2, 1, timeout_s=0.3)
    # rank 0 writes its id (and removes the file after the barrier); rank 1 reads a fresh one
    c0 = nwdist.rccl_comm(0, 2, 0)
    assert c0.rank == 0 and _FakeComm.made[-1].uid == bytes(range(128)) and not path.exists()
    path.write_bytes(bytes(range(128)))
    c1 = nwdist.rccl_comm(0, 2, 1, timeout_s=5)
    assert c1.rank == 1 and _FakeComm.made[-1].uid == bytes(range(128))
    assert nwdist.read_rendezvous_id(str(path), 1, time.time() - 10, 1) == bytes(range(128))


def test_node_records_stale_segment_is_replaced():
    """NodeRecords: rank 0 replaces a segment of the same name left by a run
    that died; publish / wait round-trips a block (world 1)."""
    import sys
    from multiprocessing import shared_memory

    sys.path.insert(0, PKG)
    import dist as nwdist

    class One:
        world, rank = 1, 0

        def max(self, x):
            return x

    key = "t%d" % os.getpid()
    stale = shared_memory.SharedMemory(name="nwk_rec_" + key, create=True, size=4096)
    stale.buf[:8] = b"\xff" * 8
    try:
        nr = nwdist.NodeRecords(One(), 2, [3, 2], key=key)
        blk = nwdist.pack_records([5, 6], [10, 11], np.full((2, 64), 9, dtype=np.uint8), 3)
        nr.publish(0, blk, 7)
        assert (nr.wait(0, 7, timeout_s=1) == blk).all()
        with pytest.raises(RuntimeError, match="not published"):
            nr.wait(1, 7, timeout_s=0.05)
        nr.close()
    finally:
        stale.close()


def test_node_stream_stale_segment_progress_and_failure():
    """NodeStream: rank 0 replaces a stale segment of the same name; progress
    words carry this call's token (an earlier call's count reads as -1), a
    publish moves the count after the records, and a failed rank's word reads
    FAILED_COUNT (world 1)."""
    import sys
    from multiprocessing import shared_memory

    sys.path.insert(0, PKG)
    import dist as nwdist

    class One:
        world, rank = 1, 0

        def max(self, x):
            return x

    key = "s%d" % os.getpid()
    stale = shared_memory.SharedMemory(name="nwk_str_" + key, create=True, size=4096)
    stale.buf[:8] = b"\xff" * 8
    try:
        ns = nwdist.NodeStream(One(), 4, key=key)
        assert list(ns.progress(1)) == [-1]  # cleared words: no record of this call yet
        blk = nwdist.pack_records([5, 6], [10, 11], np.full((2, 64), 9, dtype=np.uint8), 2)
        ns.publish(0, 2, blk, 3)
        assert list(ns.progress(3)) == [2] and list(ns.progress(4)) == [-1]
        assert (ns.take(0, 0, 2) == blk).all()
        ns.fail(4)
        assert list(ns.progress(4)) == [nwdist.NodeStream.FAILED_COUNT]
        ns.close()
    finally:
        stale.close()


def test_node_records_fast_peer_flag_survives():
    """NodeRecords: a peer may publish as soon as rank 0's nonce collective
    returns to it, before rank 0's own constructor has finished -- its flag
    must survive (rank 0 used to clear the flags after the collective, erasing
    such a flag, and then waited for it forever).  Two ranks in one process:
    rank 0's max() runs rank 1's whole attach + publish."""
    import sys

    sys.path.insert(0, PKG)
    import dist as nwdist

    key = "f%d" % os.getpid()
    blk = nwdist.pack_records([1, 2], [5, 6], np.full((2, 64), 3, dtype=np.uint8), 2)
    peer = {}

    class Peer:
        world, rank = 2, 1

        def __init__(self, nonce):
            self.nonce = nonce

        def max(self, x):
            return float(self.nonce)

    class Root:
        world, rank = 2, 0

        def max(self, x):  # the collective: the fast peer attaches and publishes piece 0 now
            peer["nr"] = nwdist.NodeRecords(Peer(int(x)), 1, [2], key=key)
            peer["nr"].publish(0, blk, 1)
            return x

    nr = nwdist.NodeRecords(Root(), 1, [2], key=key)
    try:
        nr.publish(0, blk, 1)
        got = nr.wait(0, 1, timeout_s=2)
        assert got.shape[0] == 4 and (got[2:] == blk).all()
    finally:
        peer["nr"].close()
        nr.close()
