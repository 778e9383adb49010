"""Benchmark: sequenced merge-tree ops applied per second over C3-shaped documents, with bit-exact
summaries (BASELINE.json metric).

One step = one replay of every document's op log from an empty observer Client plus its V1 summary
(Client.applyMsg for every message, then Client.summarize), i.e. mtr_reset + mtr_run + mtr_summarize.
Inputs are recorded on the device before the timed region (record mode of the engine, seeded recipe
include/mtr_synth.h), so the timed region starts with every op log resident in HBM.

Single GPU:   python bench.py
Multi GPU:    python bench.py --gpus N        (bench.py starts the N rank processes itself, one per GPU)
         or:  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
Documents are sharded over ranks.  Default strong scaling: `--docs` is the node's total (C3: 100k
documents split into contiguous equal ranges -- the LPT assignment for documents of one recipe);
`--scaling weak` gives every rank its own `--docs`.  The only collective is the final RCCL reduction of
counters and summary digests.

`value` is the device-resident rate (op logs in HBM when the timed region starts, summaries left on the
device).  The end-to-end rate SURVEY.md 8d defines -- host op upload, apply, summarize, every blob
back in host memory -- is measured separately on the same documents (`end_to_end`).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "sequenced ops applied/sec (whole node) over 100k docs, bit-exact summaries"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: chip-level parameters)
SALU_PEAK = 256 * 2.4e9  # scalar instructions per second: one SALU per CU per cycle at the 2.4 GHz peak clock


# BASELINE.json configs: documents per GPU, messages per document, writers, max lag
PRESETS = {
    # the reference's own replay logs (merge-tree/src/test/results, 30 files x 2,040 messages, 2/4/8
    # clients) as 30 documents, replayed as client.replay.spec.ts:17-71 does
    "C1": dict(docs=30, ops=2_040, writers=7, max_lag=0),
    "C2": dict(docs=10_000, ops=5_000, writers=16, max_lag=64),
    "C3": dict(docs=100_000, ops=1_000, writers=8, max_lag=32),
    # SharedMatrix replay: docs = matrices (two PermutationVector documents each), 20 % row/col
    # splices (insert 12 : remove 8) and 80 % setCell
    "C4": dict(docs=1_000, ops=20_000, writers=8, max_lag=64),
    # long context: documents pre-grown to 200,000 segments through a summary load (reloadFromSegments),
    # then collaboration with 64 writers and lags up to 4,096 (a deep window); HBM-resident
    # (1,000 documents x 20,000 messages; --docs / --ops select a part of it)
    "C5": dict(docs=1_000, ops=20_000, writers=64, max_lag=4096),
}
GROW = {"C5": 200_000}
MATRIX = {"C4"}


def host_cores_limit() -> tuple[int, str]:
    """Host cores this process may use and the limit that set it: its CPU affinity, capped by the cgroup
    CPU quota and by OMP_NUM_THREADS when the environment sets it (the GPU box gives one GPU's job a
    16-core share of a much larger machine, which os.cpu_count() does not show)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    why = f"CPU affinity mask ({n} cores)"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            q = max(1, -(-int(quota) // int(period)))
            if q < n:
                n, why = q, f"cgroup cpu.max quota {quota}/{period} ({q} cores)"
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < n:
        n, why = int(omp), f"OMP_NUM_THREADS={omp} (the job's allotment on the GPU box)"
    return max(1, n), why


def host_cores() -> int:
    return host_cores_limit()[0]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=sorted(PRESETS), default="C3",
                    help="workload preset (C3 = the headline metric's 100k-document run)")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong: --docs is the node total (split over ranks); weak: --docs per rank")
    ap.add_argument("--e2e-steps", type=int, default=2,
                    help="timed end-to-end steps (host upload -> blobs on host); 0 = skip")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--docs", type=int, default=None, help="documents: node total (strong) or per GPU (weak)")
    ap.add_argument("--ops", type=int, default=None, help="sequenced messages per document (preset)")
    ap.add_argument("--writers", type=int, default=None)
    ap.add_argument("--max-lag", type=int, default=None)
    ap.add_argument("--ops-per-launch", type=int, default=None,
                    help="ops per document per launch (48; 512 for the HBM-resident C5 documents)")
    ap.add_argument("--cpu-sample-docs", type=int, default=0,
                    help="default: about 60M messages of documents (~8 s on 16 host threads)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="default: every host core this job may use")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="multi-rank runs: nccl (= RCCL over xGMI); gloo only for the CPU tests' stub engine")
    ap.add_argument("--no-cpu-baseline", action="store_true",
                    help="skip the CPU baseline (N=1) and the per-rank oracle sample (N>1)")
    ap.add_argument("--rank-sample-docs", type=int, default=0,
                    help="N>1: documents of its own shard each rank checks against the oracle after the timed "
                         "region (default: about 4M messages' worth; one per host thread for C5)")
    ap.add_argument("--pipe-parts", type=int, default=16,
                    help="end-to-end leg: document ranges of the pipelined hand-over (mtr_replay_pipelined)")
    ap.add_argument("--master-port", type=int, default=0, help="--gpus N launcher: rendezvous port (default: a free one)")
    ap.add_argument("--traffic-file", default=None,
                    help="PMC summary of this config (default: profiles/traffic_r06_final.json for C3, traffic_r06_c5_final.json "
                         "for C5, traffic_r06_c4_final.json for C4, traffic_r06_c2_final.json for C2, traffic_r01.json "
                         "else)")
    a = ap.parse_args(argv)
    if a.traffic_file is None:
        name = {"C2": "traffic_r06_c2_final.json", "C3": "traffic_r06_final.json", "C4": "traffic_r06_c4_final.json",
                "C5": "traffic_r06_c5_final.json"}.get(
            a.config, "traffic_r01.json")
        a.traffic_file = os.path.join(ROOT, "profiles", name)
    for k, v in PRESETS[a.config].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    if a.ops_per_launch is None:
        # (C1's 30 documents are fewer than the CUs: the engine gives them launch-sized LDS room, so a launch
        # can carry a whole log -- 2,048 ops: 3.9 M ops/s against 2.4 M at 48, profiles/r04_c1_k.json)
        a.ops_per_launch = 512 if a.config in GROW else 2048 if a.config == "C1" else 48
    return a


def end_to_end(eng, n, steps, messages, matrix, hashes, barrier=lambda: None, pipe_parts=16):
    """SURVEY.md 8d's end-to-end time: the host hands the op logs over (one upload from page-locked
    memory), the engine applies and summarizes, and every blob of every document lands in host memory
    (one bulk download, mtr_get_summaries).  The op logs are the recorded ones, downloaded once
    (untimed) into pinned host memory.  Reported beside the device-resident headline, never as it."""
    import time as _t

    from fluidframework_amd.engine import pinned

    if matrix:
        return None  # (matrix pairs: the vectors' op lists are not a standalone host batch)
    t0 = _t.perf_counter()
    hb = eng.download(0, n, pinned_memory=True)
    prep_s = _t.perf_counter() - t0
    out = pinned(int(eng.summary_bytes()) + 8 * n + 4096, "u1")

    def check(what):
        if eng.stats()["bad_docs"]:
            raise SystemExit(f"end-to-end replay ({what}) left documents in an error state")
        if not np.array_equal(eng.hashes(n), hashes[:n]):
            raise SystemExit(f"end-to-end replay ({what}) produced different summaries than the device-resident steps")

    # serial hand-over: the whole upload, then apply + summarize, then the download
    times, parts = [], []
    for i in range(steps + 1):  # the first is untimed (warm)
        barrier()  # (N > 1: the ranks start each step together; the slowest rank's time is the node's)
        t0 = _t.perf_counter()
        eng.reset()
        eng.submit(hb)
        eng.sync()
        t1 = _t.perf_counter()
        eng.run()
        eng.summarize()
        eng.sync()
        t2 = _t.perf_counter()
        buf, off = eng.summaries(0, n, out=out)
        t3 = _t.perf_counter()
        if i:
            times.append(t3 - t0)
            parts.append((t1 - t0, t2 - t1, t3 - t2))
    check("serial")
    # pipelined hand-over (mtr_submit_pipelined): the op records go over in document ranges on a copy stream and
    # each range starts applying as soon as it has landed
    ptimes, pparts = [], []
    for i in range(steps + 1):
        barrier()
        t0 = _t.perf_counter()
        eng.reset()
        eng.submit_pipelined(hb, pipe_parts)
        eng.run()
        eng.summarize()
        eng.sync()
        t2 = _t.perf_counter()
        buf, off = eng.summaries(0, n, out=out)
        t3 = _t.perf_counter()
        if i:
            ptimes.append(t3 - t0)
            pparts.append((t2 - t0, t3 - t2))
    check("pipelined")
    upload_only = (float(np.mean(ptimes)), *(float(np.mean([p[q] for p in pparts])) for q in range(2)))
    # pipelined at both ends (mtr_replay_pipelined): a range whose documents are done is also summarized and its
    # records downloaded while the later ranges still upload and apply
    ptimes = []
    for i in range(steps + 1):
        barrier()
        t0 = _t.perf_counter()
        eng.reset()
        buf, off = eng.replay_pipelined(hb, out, pipe_parts)
        t3 = _t.perf_counter()
        if i:
            ptimes.append(t3 - t0)
    check("replay_pipelined")
    total = int(off[-1])
    if total != eng.summary_bytes():  # (per document: count word, lengths, blob bytes)
        raise SystemExit("bulk summary download is short")
    for d in (0, n // 2, n - 1):  # the bulk records equal the per-document reads
        if _bulk_record(buf, off, d) != eng.summary(d):
            raise SystemExit(f"bulk summary record of document {d} differs")
    t = float(np.mean(times))
    up, dev, down = (float(np.mean([p[q] for p in parts])) for q in range(3))
    tp = float(np.mean(ptimes))
    return {
        "value": round(messages / tp, 1),
        "unit": "ops/s",
        "ms_per_step": round(1000 * tp, 3),
        "parts": pipe_parts,
        "upload_pipelined": {"value": round(messages / upload_only[0], 1), "ms_per_step": round(1000 * upload_only[0], 3),
                             "upload_apply_summarize_ms": round(1000 * upload_only[1], 3),
                             "download_ms": round(1000 * upload_only[2], 3)},
        "serial": {"value": round(messages / t, 1), "ms_per_step": round(1000 * t, 3), "upload_ms": round(1000 * up, 3),
                   "apply_summarize_ms": round(1000 * dev, 3), "download_ms": round(1000 * down, 3)},
        "upload_bytes": int(hb.ops.nbytes + hb.text.nbytes + hb.docs.nbytes),
        "download_bytes": total,
        "steps": steps,
        "host_batch_prep_s": round(prep_s, 2),
        "note": "host op upload (page-locked) -> apply -> summarize -> every blob in host memory (one bulk copy); "
                "`value`: the hand-over pipelined at both ends (mtr_replay_pipelined: the records go over in `parts` "
                "document ranges on a copy stream, each range applied as soon as it lands, then summarized and its "
                "records downloaded as soon as its documents are done); `upload_pipelined`: only the upload "
                "overlapped (mtr_submit_pipelined, then summarize + one bulk download); `serial`: upload, then "
                "apply; same documents and summaries as the headline",
    }


def cpu_baseline(a, eng, n, ops, grow, matrix, hashes, fixture_batch, messages):
    """The reference's algorithm on the host cores of the same box, rank 0 at N=1:
    the oracle replays a bounded sample of the same recorded documents with one document per task on
    every host core this job may use, answering each remote block length from the block's
    PartialSequenceLengths (getPartialLength, partialLengths.ts:698-735) as the reference does.  The
    leaf-sum variant (the tests' checker) is timed on part of the sample beside it.  Both must
    reproduce the engine's summary digests."""
    from oracle.oracle import psl_answer, replay_batch, replay_matrix_batch

    threads, cores_why = host_cores_limit()
    if a.cpu_threads:
        threads, cores_why = a.cpu_threads, "--cpu-threads"
    # bounded sample: ~6e7 messages of C2/C3 documents; one pre-grown C5 document per host thread
    k = min(a.cpu_sample_docs or (threads if grow else max(1, 60_000_000 // ops)), n)
    if fixture_batch is not None:
        k = n
        sample = fixture_batch
    elif matrix:
        sample = eng.download_matrix(0, k)
    else:
        sample = eng.download(0, k)

    def replay(kk, reps=1):
        secs, oh = 0.0, None
        for _ in range(reps):
            if matrix:
                dt, oh, ost = replay_matrix_batch(sample, 0, kk, threads)
            else:
                dt, oh, ost = replay_batch(sample, 0, kk, threads)
            secs += dt / reps
        if matrix:
            eq = int((oh == hashes[:2 * kk]).reshape(kk, 2).all(axis=1).sum())
        else:
            eq = int((oh == hashes[:kk]).sum())
        return secs, eq, int((ost != 0).sum())

    reps = 10 if fixture_batch is not None else 1  # (the fixture set replays in ~0.2 s)
    with psl_answer():
        secs, eq, errs = replay(k, reps)
    bit_exact = {"checked_docs": k, "equal": eq, "oracle_errors": errs}
    if eq != k or errs:
        raise SystemExit(f"summaries differ from the CPU oracle (PartialSequenceLengths): {bit_exact}")
    k2 = k if fixture_batch is not None else max(1, k // 4)
    secs2, eq2, errs2 = replay(k2, reps)
    if eq2 != k2 or errs2:
        raise SystemExit(f"summaries differ from the CPU oracle (leaf sums): {eq2}/{k2}, {errs2} errors")
    per_doc = ops if fixture_batch is None else messages / n
    cpu = {
        "value": round(k * per_doc / secs, 1),
        "unit": "ops/s",
        "cores": threads,
        "cores_limit": cores_why,
        "kind": "port",
        "algorithm": "PartialSequenceLengths",
        "sample": f"first {k} of the {n} {'matrices' if matrix else 'documents'} ({int(k * per_doc)} messages"
                  f"{f' after {grow} loaded segments each' if grow else ''}), replay + V1 summary, one document per "
                  f"task on {threads} host threads; block lengths from PartialSequenceLengths.getPartialLength "
                  f"as in the reference (reference-algorithm C++ restatement, not Node)",
        "seconds": round(secs, 3),
        "leaf_sum": {"value": round(k2 * per_doc / secs2, 1), "docs": k2, "seconds": round(secs2, 3),
                     "note": "the oracle's leaf-sum block lengths (the tests' checker), same threads"},
        "host_cpus_visible": os.cpu_count(),
    }
    return cpu, bit_exact


def _bulk_record(buf, off, d):
    from fluidframework_amd.engine import Engine

    return Engine.split_record(buf, int(off[d]), int(off[d + 1]))


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(a, argv) -> int:
    """`--gpus N` without a launcher: start N rank processes of this script, one per GPU, and wait for them.

    The parent makes no HIP call (it imports neither torch nor the engine), so every rank initialises its own
    device from scratch.  Rank r gets RANK = LOCAL_RANK = r, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1 and a free
    MASTER_PORT, exactly what torch.distributed.run would set; rank 0 writes to this process's stdout (its JSON
    line is the run's line), the other ranks' stdout goes to stderr.  A rank that fails ends the others after a
    grace period (they would wait in a collective).  Returns the worst exit status.  The shape follows the
    reference's replay driver, which forks one worker per shard of the files and joins them
    (packages/test/snapshots/src/replayMultipleFiles.ts:355-410)."""
    import signal
    import subprocess

    port = a.master_port or _free_port()
    try:
        err_fd = sys.stderr.fileno()
    except (AttributeError, OSError, ValueError):
        err_fd = subprocess.DEVNULL
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MTR_BENCH_LAUNCHER="bench.py")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 else err_fd, start_new_session=True))
    rcs = [None] * len(procs)
    failed_at = None
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
                if rcs[i] not in (None, 0) and failed_at is None:
                    failed_at = time.time()
                    print(f"bench.py launcher: rank {i} exited with status {rcs[i]}", file=sys.stderr, flush=True)
        if failed_at is not None and time.time() - failed_at > 30:
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    os.killpg(p.pid, signal.SIGKILL)  # (the rank's own process group: start_new_session)
                    rcs[i] = p.wait()
        time.sleep(0.2)
    bad = [rc for rc in rcs if rc]
    return (bad[0] if bad[0] > 0 else 1) if bad else 0


def _engine_class():
    """The engine the bench drives: fluidframework_amd.engine.Engine (the HIP engine).  MTR_BENCH_STUB_ENGINE =
    "module:Class" substitutes a stub for the CPU tests of the multi-rank plumbing (tests/bench_stub.py); the line
    then says `"engine": "stub"`, so such a run can never pass for a measurement."""
    spec = os.environ.get("MTR_BENCH_STUB_ENGINE")
    if spec:
        import importlib

        mod, cls = spec.split(":")
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        return getattr(importlib.import_module(mod), cls), "stub"
    from fluidframework_amd.engine import Engine

    return Engine, "hip"


def rank_sample(a, eng, n, ops, grow, matrix, hashes, fixture_batch, threads):
    """N > 1: the checker leg of one rank.  After the timed region the oracle replays a bounded sample of this
    rank's own documents (the first of its shard) and compares their summary digests with the engine's; the
    counts are summed over ranks into the line's bit_exact_sample.  Not a baseline: nothing here is timed."""
    from oracle.oracle import replay_batch, replay_matrix_batch

    k = min(n, a.rank_sample_docs or (threads if grow else max(1, 4_000_000 // max(1, ops))))
    if fixture_batch is not None:
        k, sample = n, fixture_batch
    elif matrix:
        sample = eng.download_matrix(0, k)
    else:
        sample = eng.download(0, k)
    if matrix:
        _, oh, ost = replay_matrix_batch(sample, 0, k, threads)
        eq = int((oh == hashes[:2 * k]).reshape(k, 2).all(axis=1).sum())
    else:
        _, oh, ost = replay_batch(sample, 0, k, threads)
        eq = int((oh == hashes[:k]).sum())
    return {"checked_docs": int(k), "equal": eq, "oracle_errors": int((ost != 0).sum())}


def main(argv=None):
    a = parse(argv)
    if a.gpus < 1:
        raise SystemExit("--gpus must be at least 1")
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:  # no launcher around us: be it (before any HIP call)
        return launch(a, sys.argv[1:] if argv is None else argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but the launcher started {world} ranks (WORLD_SIZE): refusing to report "
                         f"a {world}-GPU run as a {a.gpus}-GPU one")
    dist = None
    reduce_device = f"cuda:{local}"
    comm_world = 1
    if world > 1:
        import torch
        import torch.distributed as dist_mod

        if a.dist_backend == "nccl":
            torch.cuda.set_device(local)
        else:
            reduce_device = "cpu"
        dist_mod.init_process_group(a.dist_backend)
        dist = dist_mod
        comm_world = dist.get_world_size()
        if comm_world != a.gpus:
            raise SystemExit(f"--gpus {a.gpus} but the process group holds {comm_world} ranks")

    from fluidframework_amd import shard
    Engine, engine_kind = _engine_class()
    from fluidframework_amd.synth import make_cfg, tables

    n, ops = a.docs, a.ops
    matrix = a.config in MATRIX
    grow = GROW.get(a.config, 0)
    tabs = tables(writers=a.writers)
    if a.scaling == "strong" and a.config != "C1":
        doc_lo, doc_hi = shard.strong_range(rank, world, n)
        n = doc_hi - doc_lo
    else:
        doc_lo, _ = shard.doc_range(rank, world, n)
    fixture_text = None
    if a.config == "C1":  # reference fixtures, not synthetic: every rank replays the same 30 logs
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from fixtures import load_replay, replay_files, replay_log

        from fluidframework_amd.batch import Interner, build_batch

        groups = [load_replay(p) for p in replay_files()]
        it = Interner()
        logs = [replay_log(g, it) for g in groups]
        for d, gs in enumerate(groups):
            for g in gs:
                for m in g["msgs"]:
                    logs[d].message(m, it)
        fixture_batch = build_batch(logs, it)
        fixture_text = [gs[-1]["resultText"] for gs in groups]
        n = len(groups)
        fixture_msgs = sum(len(g["msgs"]) for gs in groups for g in gs)
        ops = fixture_msgs // n
        eng = Engine(n, device=local, max_segments=8192, heap_entries=8192, text_units=1 << 18,
                     prop_words=1 << 18, remover_cells=1 << 14, ops_per_launch=a.ops_per_launch)
    elif matrix:
        cfg = make_cfg(n, ops, writers=a.writers, max_lag=a.max_lag, weights=(12, 8, 80), max_text=4, max_range=3,
                       doc_base=doc_lo, text_cap=0)
        # handle tables live in the text arena of a vector document (<= positions ever inserted)
        eng = Engine(2 * n, device=local, max_segments=2 * ops + 128, heap_entries=2 * ops + 128,
                     text_units=2 * ops + 1024, prop_words=1024, remover_cells=8192, ops_per_launch=a.ops_per_launch)
    elif grow:
        cfg = make_cfg(n, ops, writers=a.writers, max_lag=a.max_lag, doc_base=doc_lo,
                       text_cap=2 * grow + 18 * ops + 16)
        # (slots: the leaves plus one hole per 16 -- HBM-resident documents keep hole slots, DESIGN.md §2;
        # text: each half of the arena twice the document's text, so its collection runs rarely -- 6 MB per
        # document, 6 GB for C5's 1,000 of 288 GB)
        eng = Engine(n, device=local, max_segments=grow + grow // 14 + 2 * ops + 128, heap_entries=grow + 2 * ops + 128,
                     text_units=4 * int(cfg.text_cap) + 16384, prop_words=65536, remover_cells=65536,
                     ops_per_launch=a.ops_per_launch)
    else:
        cfg = make_cfg(n, ops, writers=a.writers, max_lag=a.max_lag, doc_base=doc_lo)
        text_units = 2 * int(cfg.text_cap) + 1024
        eng = Engine(n, device=local, max_segments=2 * ops + 128, heap_entries=2 * ops + 128, text_units=text_units,
                     prop_words=16384, remover_cells=4096, ops_per_launch=a.ops_per_launch)

    t0 = time.time()
    if fixture_text is not None:  # untimed: upload the fixture logs once (replays start from HBM)
        eng.submit(fixture_batch)
        eng.sync()
    elif matrix:  # untimed: record the op logs on the device
        eng.generate_matrix(cfg, tabs)
    else:
        eng.generate(cfg, tabs, grow=grow)
    gen_s = time.time() - t0
    gen_stats = eng.stats()
    if gen_stats["bad_docs"]:
        raise SystemExit(f"record mode left {gen_stats['bad_docs']} documents in an error state")

    def step():
        eng.reset()
        eng.run()
        eng.summarize()

    for _ in range(a.warmup):
        step()
    eng.sync()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    eng.sync()
    apply_ms = summary_ms = kernel_ms = 0.0
    launches = 0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
        tm = eng.timing()
        apply_ms += tm["apply_ms"]
        summary_ms += tm["summary_ms"]
        launches += tm["apply_launches"]
        kernel_ms += tm["apply_kernel_ms"]
    eng.sync()
    elapsed = time.perf_counter() - t0
    barrier()

    st = eng.stats()  # counters of the last step
    if fixture_text is not None:
        want = len(fixture_batch.ops)
        bad_text = sum(eng.text(d) != t for d, t in enumerate(fixture_text))
        if bad_text:
            raise SystemExit(f"{bad_text} fixture documents end with a text other than the reference's resultText")
    else:
        want = n * (grow + ops + 1)  # every document applied its whole log (loads + START_COLLAB + messages)
    if st["ops"] != want:
        raise SystemExit(f"the step applied {st['ops']} op records, expected {want}")
    hashes = eng.hashes(2 * n if matrix else n)
    messages = n * ops if fixture_text is None else fixture_msgs
    run_digest = shard.digest(hashes)
    # (after the timed region) N > 1: every rank checks a sample of its own shard against the oracle
    sample_counts = [0, 0, 0]
    if world > 1 and not a.no_cpu_baseline:
        threads = max(1, host_cores() // max(1, local_world))
        rs = rank_sample(a, eng, n, ops, grow, matrix, hashes, fixture_batch if fixture_text is not None else None,
                         threads)
        sample_counts = [rs["checked_docs"], rs["equal"], rs["oracle_errors"]]
    e2e = None
    if a.e2e_steps > 0 and fixture_text is None and not grow:
        e2e = end_to_end(eng, n, a.e2e_steps, messages, matrix, hashes, barrier=barrier, pipe_parts=a.pipe_parts)
    if dist is not None:  # the only collectives: counters + summary digests over RCCL/xGMI
        r = shard.reduce_run(dist, reduce_device, elapsed, messages, int(st["bad_docs"]), run_digest,
                             extra=sample_counts)
        elapsed, total_messages, bad, run_digest = r["elapsed"], float(r["messages"]), float(r["bad_docs"]), r["digest"]
        sample_counts = r["extra"]
        if e2e is not None:  # the slowest rank's end-to-end step times the node
            mx = shard.reduce_max(dist, reduce_device, [e2e["ms_per_step"], e2e["upload_pipelined"]["ms_per_step"],
                                                        e2e["serial"]["ms_per_step"]])
            e2e["ms_per_step"] = round(mx[0], 3)
            for k, v in (("upload_pipelined", mx[1]), ("serial", mx[2])):
                e2e[k]["ms_per_step"] = round(v, 3)
                e2e[k]["value"] = round(total_messages / (v / 1000.0), 1)
            e2e["value"] = round(total_messages / (e2e["ms_per_step"] / 1000.0), 1)
            e2e["ranks"] = world
    else:
        total_messages = float(messages)
        bad = float(st["bad_docs"])
    sample_bad = world > 1 and (sample_counts[1] != sample_counts[0] or sample_counts[2])

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        if sample_bad:
            raise SystemExit(1)
        return 0
    if sample_bad:
        raise SystemExit(f"summaries differ from the CPU oracle on the ranks' samples: {sample_counts}")

    ms_per_step = 1000.0 * elapsed / a.steps
    value = total_messages * a.steps / elapsed
    # algorithmic bytes: B_op = 16*S_d(t) + 32 + 2*L_ins, per step on this rank
    b_step = 16.0 * st["sum_leaves_before_op"] + 32.0 * messages + 2.0 * st["text_units_inserted"]
    apply_s = apply_ms / 1000.0 / a.steps
    launches_per_step = max(1, launches // a.steps)
    kernel_s = kernel_ms / 1000.0 / a.steps  # sum of the apply launches' own durations per step
    b_launch = b_step / launches_per_step
    avg_launch_s = kernel_ms / 1000.0 / max(1, launches)
    # the prescribed figure: algorithmic bytes per launch / that launch's average duration (HIP events
    # on the launch's own stream; rocprof's per-dispatch average agrees, profiles/)
    achieved = b_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    # the same bytes over the apply span: a round's size-class launches overlap on 4 streams, so the
    # span (= rocprof's first-start..last-end of the step's apply dispatches) is shorter than the sum
    achieved_span = b_step / apply_s / 1e9 if apply_s > 0 else 0.0
    traffic = pmc = None
    if os.path.exists(a.traffic_file):
        try:
            tf = json.load(open(a.traffic_file))
            if tf.get("docs") == n and tf.get("ops") == ops:
                traffic = tf.get("hbm_bytes_per_launch")
                if tf.get("hbm_bytes_per_step"):  # counted over the dominant kernel's launches of a step
                    traffic = tf["hbm_bytes_per_step"] / launches_per_step
                pmc = tf
        except (OSError, ValueError):
            traffic = pmc = None
    issue = None
    if pmc is not None:
        ipo = pmc.get("insts_per_op", {})
        issue = {
            "source": os.path.relpath(a.traffic_file, ROOT),
            "insts_per_op": round(sum(ipo.values()), 1),
            "salu_per_op": round(ipo.get("salu", 0.0), 1),
            "valu_per_op": round(ipo.get("valu", 0.0), 1),
            "lds_per_op": round(ipo.get("lds", 0.0), 1),
            "wave_cycles_waiting": round(pmc.get("wait_any_frac", 0.0), 3),
            "wave_cycles_issuing": round(pmc.get("active_inst_frac", 0.0), 3),
            "lds_bank_conflict_rate": round(pmc.get("lds_bank_conflict_rate", 0.0), 4),
            "counter_hbm_gbs": round(traffic * launches_per_step / apply_s / 1e9, 1) if traffic and apply_s > 0
            else None,
        }
        # the issue roofline of the scalar unit (one per CU, one SALU instruction per cycle: 256 CUs x 2.4 GHz),
        # which binds the replay kernels (MI355X_MICROARCH.md; SQ counters of the same build in `source`)
        salu = ipo.get("salu", 0.0)
        if salu > 0:
            per_gpu = value / max(1, world)  # (the counters are one GPU's)
            issue["salu_roofline"] = {"achieved": round(salu * per_gpu / 1e9, 1), "peak": SALU_PEAK / 1e9,
                                      "unit": "G SALU instr/s per GPU", "frac": round(salu * per_gpu / SALU_PEAK, 4)}
            clk = pmc.get("clock_ghz_measured")
            if clk:  # the same roofline at the clock the kernels ran at (GRBM_GUI_ACTIVE / 8 / duration)
                pk = SALU_PEAK / 2.4 * clk
                issue["salu_roofline"].update({"clock_ghz_nominal": 2.4, "clock_ghz_measured": round(clk, 3),
                                               "peak_measured_clock": round(pk / 1e9, 1),
                                               "frac_measured_clock": round(salu * per_gpu / pk, 4)})
    roofline = {
        "bound": "hbm",  # (the contract's vocabulary: the path's roofline is HBM; no MFMA -- what binds is in
        # `binding` and issue.salu_roofline)
        "binding": "instruction issue" if not grow else "per-wave latency",
        "limiter": "per-wave issue latency: one wave per document applies its ops in order (a chain of "
                   "dependent LDS round trips, ballots and scalar control per op); waves per SIMD are "
                   "capped by VGPRs and LDS per document. HBM sees only stage-in/out and arenas "
                   "(counter_hbm_gbs), so the HBM roofline is the flat-pass B_op model's, not the traffic's",
        "kernel": "mtr::apply_pair2_kernel" if matrix else "mtr::apply_kernel",
        "achieved": round(achieved_span, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved_span / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "per_launch": {"achieved": round(achieved, 2), "frac": round(achieved / HBM_PEAK_GBS, 4),
                       "algorithmic_bytes_per_launch": b_launch, "avg_launch_ms": kernel_ms / max(1, launches),
                       "note": "algorithmic bytes per launch / the launches' average duration (HIP events on each "
                               "launch's stream; the rocprof kernel-trace average agrees): a round's launches overlap "
                               "on 4 streams, so each runs stretched by the others and this figure double-counts "
                               "that overlap"},
        "algorithmic_bytes_per_step": b_step,
        "launches_per_step": launches_per_step,
        "apply_wall_ms_per_step": apply_ms / a.steps,
        "kernel_sum_ms_per_step": 1000.0 * kernel_s,
        "issue": issue,
        "note": "achieved / frac = the step's algorithmic bytes / the step's apply span (the driver's clock: the launches "
                "of a round overlap on 4 streams); per_launch = the same bytes per launch / the average launch "
                "duration; traffic = PMC HBM bytes per launch (2*FETCH_SIZE + WRITE_SIZE)",
        "model": "B_op = 16*S_d(t) + 32 + 2*L_ins (SURVEY.md 8d)" + (
            "; setCell: S_d = leaves of both vectors (two position resolutions)" if matrix else ""),
    }
    if grow:
        # C5: SURVEY.md 8d's two-level model is the headline (the engine's view scan is two-level: it reads
        # superchunk/chunk figures and the records of chunks with events after the op's refSeq, not every
        # leaf, so the flat-pass model would price reads it never makes and put `frac` above 1); the flat
        # figures stay beside it
        b2_step = 8.0 / 6.0 * st["sum_leaves_before_op"] + (16.0 * 14 + 32.0) * messages + 2.0 * st["text_units_inserted"]
        b2_launch = b2_step / launches_per_step
        achieved2 = b2_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
        roofline["flat_pass"] = {k: roofline[k] for k in ("model", "achieved", "frac", "per_launch",
                                                          "algorithmic_bytes_per_step")}
        a2_span = b2_step / apply_s / 1e9 if apply_s > 0 else 0.0
        roofline.update({
            "model": "B_op2 = 8*#blocks + 16*(leaf records in <= 2 touched leaf blocks) + 32 + 2*L_ins; "
                     "#blocks ~ S/6 (reloadFromSegments' 7-per-block layout and its splits), 2 leaf blocks = 14 "
                     "records (SURVEY.md 8d, two-level)",
            "achieved": round(a2_span, 2),
            "frac": round(a2_span / HBM_PEAK_GBS, 4),
            "per_launch": {"achieved": round(achieved2, 2), "frac": round(achieved2 / HBM_PEAK_GBS, 4),
                           "algorithmic_bytes_per_launch": b2_launch, "avg_launch_ms": kernel_ms / max(1, launches)},
            "algorithmic_bytes_per_step": b2_step,
            "limiter": "per-document latency: a two-wave workgroup per document (wave 0 applies the ops in order, "
                       "wave 1 takes halves of the view scan's superchunk rounds, the dirty-chunk evaluation, the "
                       "block walks and packParent), each op a chain of dependent HBM round trips (superchunk/chunk "
                       "figures in LDS, records of chunks with later events, the op's leaf region) and scalar "
                       "control; the scalar unit is shared by the CU's waves",
        })

    cpu = None
    bit_exact = {"checked_docs": 0, "equal": 0}
    if world > 1:
        bit_exact = {"checked_docs": sample_counts[0], "equal": sample_counts[1], "oracle_errors": sample_counts[2],
                     "ranks": world, "note": "each rank replayed the first documents of its own shard on the oracle "
                                             "after the timed region; counts summed over ranks"}
    if not a.no_cpu_baseline and world == 1:
        cpu, bit_exact = cpu_baseline(a, eng, n, ops, grow, matrix, hashes, fixture_batch if fixture_text is not None
                                      else None, messages)
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "ops/s",
        "n_gpus": world,
        "rccl_world_size": comm_world if dist is not None else None,
        "launcher": os.environ.get("MTR_BENCH_LAUNCHER", "torch.distributed.run" if world > 1 else None),
        "engine": engine_kind,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": a.scaling if a.config != "C1" else "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": ("reference fixtures (tests/golden/replay, converted from merge-tree/src/test/results)"
                 if fixture_text is not None else
                 "synthetic: seeded recipe include/mtr_synth.h recorded on the device (record mode)"),
        "config": {
            "workload": (f"C1: the reference's 30 replay logs (merge-tree/src/test/results) as {n} documents, "
                         f"{messages} sequenced messages (plus initial text + startOrUpdateCollaboration), final texts "
                         f"checked against resultText, V1 summaries" if fixture_text is not None else
                         f"{a.config}: {n} SharedMatrix docs/GPU (2 PermutationVectors each) x {ops} ops, 20% row/col "
                         f"splices + 80% setCell, {a.writers} writers, lag<={a.max_lag}, V1 segments + handleTable"
                         if matrix else
                         f"{a.config}: {n} docs/GPU ({a.docs} {'per GPU' if a.scaling == 'weak' else 'in all'}) x {ops} ops, "
                         f"{a.writers} writers, lag<={a.max_lag}, V1 summaries"
                         + (f", each pre-grown to {grow} segments by a summary load (HBM-resident)" if grow else "")),
            "docs_per_gpu": n,
            "docs_total": int(n * world) if a.scaling == "weak" or a.config == "C1" else int(a.docs),
            "ops_per_doc": ops,
            "writers": a.writers,
            "max_lag": a.max_lag,
            "parallelism": f"doc-sharded x{world} ({a.scaling if a.config != 'C1' else 'replicas'})",
        },
        "roofline": roofline,
        "end_to_end": e2e,
        "cpu_baseline": cpu,
        "bit_exact_sample": bit_exact,
        "detail": {
            "apply_ms_per_step": round(apply_ms / a.steps, 3),
            "summary_ms_per_step": round(summary_ms / a.steps, 3),
            "summary_bytes": eng.summary_bytes(),
            "bad_docs": int(bad),
            "digest": f"{run_digest:016x}",
            "generate_s": round(gen_s, 2),
            "max_leaves": st["max_leaves"],
            "max_heap": st["max_heap"],
            "mean_leaves_before_op": st["sum_leaves_before_op"] / max(1, messages),
        },
    }
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main() or 0)
