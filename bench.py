#!/usr/bin/env python3
"""Benchmark: all-pairs Needleman-Wunsch on MI355X, reference metric GCUPS.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|big13|c4|c5]

One "step" = the whole getMinimumPenalties job of the workload (skel:117-175,
sub:232-364): every pair's fill + traceback + trim + SHA-512 on its rank's GPU,
the ONE all-gather of 72-byte result records across ranks (N>1, RCCL), and
rank 0's hash chain.  Sequences are resident in HBM before the timed region.
value = total DP cells of the job / max-over-ranks wall time per step (strong
scaling: the workload is fixed, its pairs are LPT-sharded over N GPUs).

Default workload = C3 (BASELINE.json configs[2]), the configuration the
north_star target is quoted on: synthetic k=64, L=50,000 ACGT, pxy=3 pgap=2,
2,016 pairs, 5.04e12 cells.  Its answer hash and penalties are checked in-run
against tests/golden/large/c3.json (oracle/_ref/sub, the reference's own
program compiled from its sources, run in the build container).  big13 is
checked against the reference's published answer (testing3/sequential.txt).

--gpus N without torch.distributed.run: the bench launches N rank processes
itself (before anything touches the GPU) and fails if N exceeds the visible
devices; under torch.distributed.run, --gpus must equal WORLD_SIZE.

Also reported (rank 0):
  roofline      the fill kernel (99.5% of GPU time).  Its per-launch duration
                is measured live (HIP events on the engine stream).  Its
                per-launch counters -- VALU wave-instructions, GRBM_GUI_ACTIVE,
                HBM bytes (2 x FETCH_SIZE + WRITE_SIZE) -- come from the
                rocprofv3 --pmc passes of this same command committed under
                profiles/<round>/pmc_<workload>.json (tools/pmc_roofline.py).
                frac is <= 1 for both roofs; "bound" names the larger.
  cpu_baseline  the reference's submitted MPI+OpenMP program (oracle/_ref/sub,
                compiled from the reference sources) under mpirun on this
                host, on a labelled prefix subset of the same workload.
"""
import argparse
import glob
import json
import os
import shutil
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd")
ORACLE = os.path.join(REPO, "oracle")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

import workloads  # noqa: E402

METRIC = "DP cell-updates/s (GCUPS) on k-way SoP MSA; 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E ~8 TB/s
SIMDS = 1024                   # 256 CUs x 4 SIMDs
VALU_CYC_PER_WAVE_INSTR = 2    # MI355X_MICROARCH.md: a wave64 VALU instruction issues over 2 cycles
SPEC_CLOCK_HZ = 2.4e9          # MI355X_MICROARCH.md: peak engine clock (the spec-clock roofline)
BYTES_PER_CELL = 4.0           # the reference's int32 matrix (sub:428, 478-487)
GOLDEN = os.path.join(REPO, "tests", "golden")


def load_workload(name):
    """(description, pxy, pgap, genes, affine, expected answer or None)."""
    import seqalign

    if name == "big13":
        text = open(os.path.join(GOLDEN, "data", "mseq-big13-example.txt"), "rb").read()
        pxy, pgap, genes = seqalign.parse_input(text)
        gold = {c["name"]: c for c in json.load(open(os.path.join(GOLDEN, "golden.json")))["cases"]}
        g = gold["big13"]
        return "mseq-big13-example.txt (k=13)", pxy, pgap, genes, None, {
            "hash": g["hash"], "penalties": g["penalties"], "source": g["source"]}
    if name in workloads.SYNTH:
        desc, k, L, pxy, pgap, affine = workloads.SYNTH[name]
        expect = None
        f = os.path.join(GOLDEN, "large", name + ".json")
        if os.path.exists(f) and affine is None:
            g = json.load(open(f))
            expect = {"hash": g["hash"], "penalties": g["penalties"], "source": g["source"]}
        fa = os.path.join(GOLDEN, "large", name + "_pen.json")
        if affine is not None and os.path.exists(fa):
            # the affine variant has no reference: every penalty
            # against the oracle's O(n)-memory Gotoh scorer, no answer hash
            g = json.load(open(fa))
            expect = {"hash": None, "penalties": g["penalties"], "source": g["source"],
                      "affine": (g["go"], g["ge"])}
        return desc, pxy, pgap, workloads.synth(k, L), affine, expect
    raise SystemExit("unknown workload " + name)


# ---------------------------------------------------------------------------
# CPU baseline: the reference's own program on this host
# ---------------------------------------------------------------------------
def host_info():
    info = {"host_cpus": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except Exception:
        pass
    try:
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        if q[0] != "max":
            info["cgroup_cpu_quota"] = round(int(q[0]) / int(q[1]), 2)
    except Exception:
        pass
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")]
        sockets = {l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("physical id")}
        info["cpu_model"] = model[0] if model else None
        info["sockets"] = len(sockets) or None
    except Exception:
        pass
    return info


def cpu_share():
    """CPUs this run may use: the box gives one GPU's job a 16-CPU share
    (OMP_NUM_THREADS=16 there); a cgroup quota or affinity mask below that wins."""
    share = int(os.environ.get("NWK_BENCH_CPU_SHARE", os.environ.get("OMP_NUM_THREADS", "16")) or 16)
    hi = host_info()
    for key in ("affinity_cpus", "cgroup_cpu_quota"):
        if hi.get(key):
            share = min(share, int(hi[key]))
    return max(share, 1), hi


def _run_beating(cmd, data, timeout, tag):
    """subprocess.run(cmd, input=data) that prints a heartbeat to stderr every 30 s
    (a GPU-box command silent for 3 minutes is taken to be hung)."""
    import threading

    p = subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    res = {}
    th = threading.Thread(target=lambda: res.update(zip(("out", "err"), p.communicate(data))))
    th.start()
    t0 = time.perf_counter()
    while th.is_alive():
        th.join(30)
        if th.is_alive():
            if time.perf_counter() - t0 > timeout:
                p.kill()
                th.join()
                raise subprocess.TimeoutExpired(cmd, timeout)
            print("%s: running %.0f s" % (tag, time.perf_counter() - t0), file=sys.stderr, flush=True)
    return subprocess.CompletedProcess(cmd, p.returncode, res.get("out", b""), res.get("err", b""))


def cpu_baseline(genes, pxy, pgap, affine=None, budget_s=60.0, expect_pen=None, expect_hs=None):
    """The CPU path on a bounded prefix subset of the workload (>= 60 s, the
    depth BASELINE.md §3 asks for: "the first P' pairs in canonical order, with
    P' chosen for >= 60 s").

    linear: the reference's submitted program (oracle/_ref/sub, compiled from
    submit/xuliny-seqalkway.cpp), R = share // 16 MPI ranks under mpirun (sub
    hard-codes 16 OpenMP threads per rank, sub:94,238,425), on the first k'
    sequences of the workload -- exactly its first k'(k'-1)/2 canonical pairs
    -- with k' the smallest whose estimated time at the reference's measured
    ~0.06 GCUPS/core reaches budget_s (whole workloads shorter than that run in full).
    affine: the reference has no affine path, so the oracle's restatement
    (single thread, O(n) score-only fill) on one pair cut to fit the budget.

    expect_pen / expect_hs: the job's canonical penalties and raw problem
    hashes (the GPU's, whose full answer was checked against the reference):
    sub's printed answer for its prefix must equal their first k'(k'-1)/2
    entries and the chain over them (answer_ok).  sub has a data race in its
    master region (sub:242, 272-285: the shared task_id) that can garble its
    answer; a garbled run is re-run once, and both outcomes are reported.
    """
    import oracle

    share, hi = cpu_share()
    if affine:
        go, ge = affine
        L = int((budget_s * 0.25e9) ** 0.5)
        x, y = genes[1][:L], genes[0][:L]
        t0 = time.perf_counter()
        oracle.score_affine(x, y, pxy, go, ge)
        dt = time.perf_counter() - t0
        return dict({"value": round(len(x) * len(y) / dt / 1e9, 4), "unit": "GCUPS", "cores": 1, "kind": "port",
                     "sample": "oracle nwo_score_affine (1 thread, score-only) on pair (1,0) cut to %d x %d" % (
                         len(x), len(y))}, **hi)
    ranks = max(1, share // 16)
    est_gcups = 0.06 * 16 * ranks
    L = np.array([len(g) for g in genes], dtype=np.float64)
    kk = 2
    while kk < len(genes) and workloads.cells(genes[:kk]) / (est_gcups * 1e9) < budget_s:
        kk += 1
    sample = genes[:kk]
    cells = workloads.cells(sample)
    text = workloads.token_text(pxy, pgap, sample)
    desc = "first %d sequences of the workload (canonical pairs 0..%d, lengths %d-%d), %.3g cells" % (
        kk, kk * (kk - 1) // 2 - 1, int(L[:kk].min()), int(L[:kk].max()), cells)
    sub = os.path.join(oracle.REF_DIR, "sub")
    mpirun = shutil.which("mpirun") or ("/opt/conda/bin/mpirun" if os.path.exists("/opt/conda/bin/mpirun") else None)
    if os.path.exists(sub):
        cmd = [sub] if ranks == 1 or mpirun is None else [mpirun, "-np", str(ranks), sub]
        try:
            Pk = kk * (kk - 1) // 2
            want = None
            if expect_pen is not None and expect_hs is not None:
                import seqalign

                want = (seqalign.chain_hash(np.asarray(expect_hs)[:Pk]), [int(v) for v in expect_pen[:Pk]])
            runs = []
            for attempt in range(2):
                r = _run_beating(cmd, text, 900, "cpu_baseline (reference sub, attempt %d)" % (attempt + 1))
                if r.returncode != 0:
                    raise RuntimeError("exit %d: %s" % (r.returncode, r.stderr[-300:].decode("latin-1")))
                lines = r.stdout.decode("latin-1").split("\n")
                ti = max(i for i, l in enumerate(lines) if l.startswith("Time: "))
                us = int(lines[ti].split()[1])
                got_h = lines[ti + 1].strip()
                got_p = [int(v) for v in lines[ti + 2].split()] if len(lines) > ti + 2 else []
                ok = None if want is None else (got_h == want[0] and got_p == want[1])
                runs.append({"us": us, "answer_hash": got_h, "answer_ok": ok})
                if ok is not False:
                    break
            us = runs[-1]["us"]
            return dict({"value": round(cells / us / 1e3, 4), "unit": "GCUPS", "cores": 16 * ranks,
                         "kind": "reference", "ranks": ranks,
                         "launch": " ".join(os.path.basename(c) for c in cmd),
                         "sample": "oracle/_ref/sub (submit/xuliny-seqalkway.cpp, %d rank(s) x 16 OpenMP threads; "
                                   "CPU share of this run = %d) on %s" % (ranks, share, desc),
                         "answer_hash": runs[-1]["answer_hash"], "answer_ok": runs[-1]["answer_ok"],
                         "answer_checked_against": None if want is None else
                         "the first %d canonical penalties and the chain over their problem hashes from this "
                         "run's GPU answer (itself checked against the reference)" % Pk,
                         "runs": len(runs), "garbled_runs": sum(1 for x in runs if x["answer_ok"] is False)}, **hi)
        except Exception as e:  # fall through to the port
            desc += " [reference binary failed: %s]" % str(e)[:160]
    # port: the oracle CLI (single-thread restatement of skel) on the 3 first, cut to 20k
    sample = [g[:20000] for g in genes[:3]]
    cells = workloads.cells(sample)
    us, _, _ = oracle.run_cli(oracle.CLI, workloads.token_text(pxy, pgap, sample), timeout=600)
    return dict({"value": round(cells / us / 1e3, 4), "unit": "GCUPS", "cores": 1, "kind": "port",
                 "sample": "oracle/_build/nw_oracle (skel restatement, 1 thread) on 3 sequences cut to 20000 "
                           "(%.3g cells); %s" % (cells, desc)}, **hi)


# ---------------------------------------------------------------------------
# Roofline: live kernel duration x committed per-launch counters
# ---------------------------------------------------------------------------
def load_pmc(workload, kernel):
    """Newest profiles/r*/pmc_<workload>.json for this kernel (per-launch counters)."""
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "pmc_%s.json" % workload)), reverse=True):
        d = json.load(open(f))
        if d.get("kernel", "").endswith(kernel):
            d["_file"] = os.path.relpath(f, REPO)
            return d
    return None


def roofline(workload, kernel, launch_s, my_cells, launches):
    import seqalign

    pmc = load_pmc(workload, kernel)
    sid = seqalign.kernel_source_id(kernel)
    eq_gbs = my_cells * BYTES_PER_CELL / launches / launch_s / 1e9
    out = {"kernel": kernel, "launch_ms": round(launch_s * 1e3, 3),
           "equivalent_4B_per_cell_GBps": round(eq_gbs, 1), "kernel_source_id": sid}
    note = None
    if pmc is None:
        note = "no profiles/r*/pmc_%s.json for %s" % (workload, kernel)
    elif pmc.get("kernel_source_id") != sid:
        note = ("%s holds counters of kernel build %s, this run's %s is %s: no counter roofline until the "
                "PMC passes are re-run on this build" % (pmc["_file"], pmc.get("kernel_source_id"), kernel, sid))
    if note:
        out.update({"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None,
                    "note": note})
        return out
    clk = pmc["grbm_gui_active_per_launch"] / 8.0 / (pmc["duration_ns_per_launch"] * 1e-9)  # Hz, 8 XCDs
    insts = pmc["sq_insts_valu_per_launch"]
    valu_frac = insts * VALU_CYC_PER_WAVE_INSTR / SIMDS / (clk * launch_s)
    # (the guide's peak clock: frac_spec_clock prices the same issue against 2.4 GHz,
    # "frac" against the clock the counters measured -- both reported)
    valu_frac_spec = insts * VALU_CYC_PER_WAVE_INSTR / SIMDS / (SPEC_CLOCK_HZ * launch_s)
    valu = {"achieved": round(insts * 64 / launch_s / 1e12, 2),
            "peak": round(SIMDS * 64 / VALU_CYC_PER_WAVE_INSTR * clk / 1e12, 2),
            "unit": "Tlane-op/s", "frac": round(valu_frac, 4), "clock_GHz": round(clk / 1e9, 3),
            "peak_spec_clock": round(SIMDS * 64 / VALU_CYC_PER_WAVE_INSTR * SPEC_CLOCK_HZ / 1e12, 2),
            "frac_spec_clock": round(valu_frac_spec, 4), "spec_clock_GHz": SPEC_CLOCK_HZ / 1e9,
            "valu_wave_instr_per_launch": insts}
    traffic = pmc["hbm_bytes_per_launch"]
    hbm = {"achieved": round(traffic / launch_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(traffic / launch_s / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic}
    bound = "valu" if valu["frac"] >= hbm["frac"] else "hbm"
    top = valu if bound == "valu" else hbm
    out.update({"bound": bound, "achieved": top["achieved"], "peak": top["peak"], "unit": top["unit"],
                "frac": top["frac"], "frac_clock": "measured" if bound == "valu" else None,
                "frac_spec_clock": valu["frac_spec_clock"] if bound == "valu" else top["frac"],
                "traffic": traffic, "valu": valu, "hbm": hbm,
                "counters_from": pmc["_file"] + " (rocprofv3 --pmc passes of this bench command; "
                                 "duration measured live here, counters per launch from the passes)"})
    return out


# ---------------------------------------------------------------------------
# Rank launcher for `bench.py --gpus N` outside torch.distributed.run
# ---------------------------------------------------------------------------
def spawn_ranks(n):
    share = os.environ.get("NWK_BENCH_SHARE_GPU") == "1"
    if not share:
        import torch  # device_count() does not initialise the GPU on this image

        vis = torch.cuda.device_count()
        if n > vis:
            print("bench.py: --gpus %d but only %d GPU(s) visible" % (n, vis), file=sys.stderr)
            return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    run_id = os.urandom(8).hex()  # names this launch's rendezvous files / shared memory (dist.run_key)
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NWK_RUN_ID=run_id)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    return wait_ranks(procs)


def wait_ranks(procs, poll_s=0.05, grace_s=10.0):
    """Waits for every rank process.  The first non-zero exit (in time, not in
    rank order -- a peer blocked in init_process_group or the all-gather would
    otherwise hold the launcher) terminates the others, then kills what is left
    after grace_s; every child is reaped.  Returns that first failure code, or 0."""
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
                t_end = time.time() + grace_s
                for q in live:
                    try:
                        q.wait(timeout=max(0.0, t_end - time.time()))
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                live = []
                break
        if live:
            time.sleep(poll_s)
    return rc


def mapped_libs():
    keys = ("libamdhip64", "librccl", "libhsa-runtime64", "libnwk")
    libs = set()
    try:
        for line in open("/proc/self/maps"):
            path = line.split()[-1] if len(line.split()) >= 6 else ""
            if any(k in os.path.basename(path) for k in keys):
                libs.add(path)
    except OSError:
        pass
    return sorted(libs)


def nwdist_auto_chunks(P, world):
    import dist as nwdist

    return nwdist.auto_chunks(P, world)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="c3", choices=["c3", "big13", "c4", "c5"])
    ap.add_argument("--bits", type=int, default=0, help="force DP storage width (4/8/16/32)")
    ap.add_argument("--affine", default=None,
                    help="go,ge: run the affine-gap variant (default for --workload c5: 3,1)")
    ap.add_argument("--kernel", default="auto",
                    help="linear fill kernel (seqalign.Engine.KERNEL): auto, nw_align_bits, nw_align_col, ...")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import seqalign

    comm = None
    gpu = local
    # NWK_BENCH_FORCE_DIST=1 (tests): the sharded path -- communicator, LPT
    # shard, the all-gathers -- even at WORLD_SIZE 1, so a 1-GPU box runs the
    # RCCL collective the driver's N-GPU runs use
    sharded = world > 1 or os.environ.get("NWK_BENCH_FORCE_DIST") == "1"
    if sharded:
        import dist as nwdist

        # Test hooks (not used by the driver): NWK_BENCH_BACKEND=gloo and
        # NWK_BENCH_SHARE_GPU=1 run the N-rank path on a 1-GPU box.
        backend = os.environ.get("NWK_BENCH_BACKEND", "nccl")
        ndev = seqalign.device_count()
        if os.environ.get("NWK_BENCH_SHARE_GPU") == "1":
            gpu = local % max(1, ndev)
        elif local >= ndev:
            sys.exit("bench.py: rank %d has no GPU (%d visible)" % (local, ndev))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            # RCCL through the library (nwk_comm_*): this process maps one HIP
            # runtime and one RCCL, the library's -- torch is never imported here
            comm = nwdist.rccl_comm(gpu, world, rank)
        else:
            import torch.distributed as tdist

            tdist.init_process_group(backend)
            comm = nwdist.TorchComm()
        world = comm.world  # n_gpus comes from the communicator

    name, pxy, pgap, genes, affine, expect = load_workload(args.workload)
    if args.affine is not None:
        affine = tuple(int(v) for v in args.affine.split(","))
    if affine and tuple(affine) != (0, pgap) and (expect is None or tuple(expect.get("affine", ())) != tuple(affine)):
        expect = None  # the reference's answers are for linear gaps (== affine go=0, ge=pgap only)
    elif affine and expect is not None and "affine" in expect and tuple(affine) == (0, pgap):
        expect = None  # (an affine fixture's penalties are not the linear run's)
    if affine:
        go, ge = affine
    k = len(genes)
    P = k * (k - 1) // 2
    lengths = [len(g) for g in genes]
    total_cells = workloads.cells(genes)
    ws = int(float(os.environ.get("NWK_BENCH_WS_GB", "0")) * (1 << 30))  # test hook: per-rank HBM budget
    # sharded linear jobs of many pairs (C4: 32,640, a ~14 ms chain on rank 0):
    # one launch per rank whose records stream out as pairs are hashed inside
    # the fill launch (finalize "fused"), pieces of canonical ids exchanged and
    # chained as they complete (C4 at 8 ranks: 24.3 ms vs 28.4 ms)
    stream = sharded and not affine and int(os.environ.get("NWK_BENCH_STREAM", "1" if P >= 8192 else "0")) == 1
    eng = seqalign.Engine(device=gpu, bits=args.bits, verbose=args.verbose, workspace_bytes=ws,
                          finalize="fused" if stream else "auto", kernel=args.kernel)
    eng.set_sequences(genes)  # sequences resident in HBM before timing
    my_ids = seqalign.shard_pairs(lengths, rank, world) if sharded else np.arange(P, dtype=np.int64)

    if affine:
        def align(ids, a, b):
            return eng.align_pairs_affine(ids, a, go, ge)
    else:
        align = eng.align_pairs

    # sharded linear runs: the shard in `chunks` pieces, each piece's records
    # all-gathered (and chained on rank 0) while the next piece aligns
    chunks = int(os.environ.get("NWK_BENCH_CHUNKS", "0")) or (16 if stream else nwdist_auto_chunks(P, world))
    # streamed jobs with every rank on this node: the pieces' records reach rank
    # 0's chain through shared memory as they stream out of each rank's launch,
    # and the whole shard's records go through ONE RCCL all-gather after it (an
    # RCCL kernel cannot start while the persistent fill holds every SIMD's
    # registers: dist.NodeRecords).  NWK_NODE_RECORDS=0: one
    # all-gather per piece instead.
    # Since round 6 the records go one at a time (NWK_BENCH_RECORDS=1, the
    # default: dist.NodeStream, rank 0's chain takes each record as soon as its
    # rank has published it); NWK_BENCH_RECORDS=0 keeps the 16 pieces.
    node = None
    per_record = False
    if stream and nwdist.node_local(world) and os.environ.get("NWK_NODE_RECORDS", "1") != "0":
        per_record = os.environ.get("NWK_BENCH_RECORDS", "1") != "0"
        if per_record:
            node = nwdist.NodeStream(comm, nwdist.stream_per(lengths, world))
        else:
            node = nwdist.NodeRecords(comm, chunks, nwdist.chunk_parts(lengths, rank, world, chunks)[1])
    token = [0]
    piece_stats = []
    last_hs = [None]
    piece_t = []  # per piece: ms from the step's start until its records were ready on this rank

    def step():
        del piece_stats[:]
        del piece_t[:]
        hs = None
        t_step = time.perf_counter()
        if per_record:
            token[0] += 1
            h, pen, hs = nwdist.align_sharded_records(
                eng, lengths, pxy, pgap, rank, world, node, token[0], comm=comm,
                on_first=lambda: piece_t.append(round((time.perf_counter() - t_step) * 1e3, 3)))
            piece_stats.append(eng.stats())
        elif stream:
            token[0] += 1
            h, pen, hs = nwdist.align_sharded_streamed(
                eng, lengths, pxy, pgap, rank, world, chunks=chunks, comm=comm, node=node, token=token[0],
                on_piece=lambda c: piece_t.append(round((time.perf_counter() - t_step) * 1e3, 3)))
            piece_stats.append(eng.stats())  # (the call has ended inside)
        elif sharded and not affine:
            h, pen, hs = nwdist.align_sharded_pipelined(eng, lengths, pxy, pgap, rank, world, chunks=chunks,
                                                       comm=comm,
                                                       on_piece=lambda c: (piece_stats.append(eng.stats()),
                                                                           piece_t.append(round(
                                                                               (time.perf_counter() - t_step) * 1e3,
                                                                               3))))
        elif sharded:
            pen, hs, _ = nwdist.align_sharded(align, lengths, pxy, pgap, rank, world, comm=comm)
            h = seqalign.chain_hash(hs) if rank == 0 else None
            piece_stats.append(eng.stats())
        else:  # getMinimumPenalties on the engine: the chain overlaps later batches
            h, pen, hs = eng.align_all(pxy, pgap, affine=(go, ge) if affine else None)
            piece_stats.append(eng.stats())
        last_hs[0] = hs
        return pen, h

    def sync():
        if sharded:
            comm.barrier()
            seqalign.device_synchronize(gpu)

    def check(pen, h):
        if rank != 0 or expect is None:
            return None
        return (expect["hash"] is None or h == expect["hash"]) and [int(v) for v in pen] == expect["penalties"]

    checks = []
    for _ in range(args.warmup):
        checks.append(check(*step()))
    sync()
    fills, traces = [], []
    t0 = time.perf_counter()
    launches = 0
    for _ in range(args.steps):
        pen, h = step()
        fills.append(sum(x["fill_ms"] for x in piece_stats))
        traces.append(sum(x["traceback_ms"] for x in piece_stats))
        launches = sum(x["fill_launches"] for x in piece_stats)
    sync()
    dt = time.perf_counter() - t0
    checks.append(check(pen, h))  # the last timed step's answer
    if sharded:
        dt = comm.max(dt)  # the slowest rank's time
    if rank != 0:
        eng.close()
        if node is not None:
            node.close()
        comm.close()
        return

    ms_step = dt / max(args.steps, 1) * 1e3
    gcups = total_cells * args.steps / dt / 1e9
    st = eng.stats()
    my_cells = workloads.cells(genes, my_ids) if sharded else total_cells
    fill_ms = float(np.mean(fills)) if fills else float("nan")
    launches = max(launches, 1)
    kernel = seqalign.KERNELS.get(st["mode"], "?")
    answer_ok = None if expect is None else all(c is True for c in checks)
    out = {
        "metric": METRIC,
        "value": round(gcups, 3),
        "unit": "GCUPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int16x2-relative (int32-exact results, 4-bit mod-16 traceback storage)"
                 if st["mode"] in (4, 5) else
                 "int16x2-relative, x4 with 2-bit source tags (int32-exact results, 4-bit traceback codes)"
                 if st["mode"] == 7 else
                 "u32 bit planes (bit-sliced: 32 cells per VALU op, 2*pgap thermometer planes of the "
                 "G-space differences; int32-exact results, 2-bit traceback storage)"
                 if st["mode"] in (8, 9, 10) else
                 "u32 bit planes (bit-sliced Gotoh: 32 cells per VALU op, 2(go+ge) difference and go gap-offset "
                 "thermometer planes; int32-exact results, 4 traceback bits per cell)"
                 if st["mode"] == 11 else ("int32" if st["bits"] == 32 else
                                              "int32 (%d-bit mod-2^W traceback storage)" % st["bits"]),
        "data": "reference input file (mseq-big13-example.txt)" if args.workload == "big13"
                else "synthetic (seeded MT19937 ACGT, workloads.py)",
        "config": {"workload": name, "pairs": P, "cells": total_cells, "pxy": pxy,
                   "gaps": ("affine go=%d ge=%d" % (go, ge)) if affine else "linear pgap=%d" % pgap,
                   "storage_bits_per_cell": st["bits"], "mode": seqalign.MODES.get(st["mode"]),
                   "parallelism": "pair-sharded dp%d (LPT), %d all-gather(s) of 72-B records, chain streamed on rank 0%s" % (
                       world, chunks if sharded and not affine and node is None else 1,
                       "; one launch per rank, records streamed per pair (fused device finalize)" if stream else "")},
        "answer_hash_ok": answer_ok,
        "answer_source": expect["source"] if expect else None,
        "answer_checked": None if expect is None else (
            "all %d penalties (no reference hash for the affine variant)" % P if expect["hash"] is None
            else "answer hash + all %d penalties" % P),
        "kernel": {"name": kernel, "fill_ms": round(fill_ms, 3), "traceback_ms": round(float(np.mean(traces)), 3),
                   "fill_gcups": round(my_cells / (fill_ms * 1e-3) / 1e9, 2),
                   "fill_launches_per_step": launches, "batches": sum(x["batches"] for x in piece_stats),
                   "window_retries": sum(x.get("window_retries", 0) for x in piece_stats),
                   "window": st.get("window", 0)},
        "roofline": roofline(args.workload if not args.affine else args.workload + "_affine", kernel,
                             fill_ms / launches * 1e-3, my_cells, launches),
    }
    if sharded:
        out["collective"] = {"backend": comm.backend,
                             "all_gathers_per_step": 1 if affine or node is not None else chunks,
                             "piece_exchange": "every record through node shared memory as it is out "
                                               "(dist.NodeStream), then one all-gather" if per_record else
                                               "node shared memory (dist.NodeRecords), then one all-gather"
                                               if node is not None else "one all-gather per piece",
                             "record_bytes": 72, "forced_at_world_1": world == 1,
                             "pieces_per_rank": "per record" if per_record else 1 if affine else chunks,
                             # rank 0, last timed step: when its chain took the first record
                             # (per record), or when each piece's records were ready
                             ("first_record_ms" if per_record else "piece_ready_ms"): list(piece_t)}
    # which HIP runtime / RCCL this process bound (torch, when imported first,
    # brings its own libamdhip64 / librccl and libnwk.so binds to those)
    out["runtime_libs"] = mapped_libs()
    if not args.no_cpu_baseline and world == 1:
        ok_gpu = answer_ok is True
        out["cpu_baseline"] = cpu_baseline(genes, pxy, pgap, affine, expect_pen=pen if ok_gpu else None,
                                           expect_hs=last_hs[0] if ok_gpu else None)
    print(json.dumps(out), flush=True)
    eng.close()
    if node is not None:
        node.close()
    if comm is not None:
        comm.close()
    if answer_ok is False:
        sys.exit("bench.py: answer hash / penalties differ from " + expect["source"])


if __name__ == "__main__":
    main()
