"""bench.py's multi-rank branch (world > 1) on CPU: two ranks over gloo, each replaying its strong-scaling
document range, then shard.reduce_run's all-reduces and rank 0's JSON line.

The engine is stubbed at its Python ABI wrapper (fluidframework_amd.engine.Engine): the stub records
and "replays" its documents with the CPU oracle as the checker (test infrastructure only), so the
counters, digests and timing the bench reduces are real.  What is checked: the line's message total,
the digest (it must equal a single-process digest over all documents), n_gpus, and that the timed
region's max over ranks is what `value` divides by.
"""
import io
import json
import os
import socket
import sys
from contextlib import redirect_stdout

import numpy as np
import subprocess

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
DOCS, OPS = 5, 90  # node total (strong scaling): ranks hold 3 and 2 documents


from bench_stub import StubEngine  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench
    import fluidframework_amd.engine as engine_mod
    engine_mod.Engine = StubEngine
    buf = io.StringIO()
    with redirect_stdout(buf):
        bench.main(["--gpus", str(world), "--docs", str(DOCS), "--ops", str(OPS), "--writers", "4", "--max-lag", "8",
                    "--steps", "3", "--warmup", "1", "--dist-backend", "gloo", "--traffic-file", "/nonexistent",
                    "--e2e-steps", "0"])
    q.put((rank, buf.getvalue()))


def test_bench_two_ranks_gloo_stub_engine():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert outs[1].strip() == ""  # only rank 0 prints
    line = json.loads(outs[0].strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["steps"] == 3 and line["scaling"] == "strong"
    assert line["config"]["docs_total"] == DOCS and line["config"]["docs_per_gpu"] == 3  # rank 0's range
    # value = every rank's messages over the max-over-ranks elapsed time
    assert abs(line["value"] * line["ms_per_step"] / 1000.0 - DOCS * OPS) < 1e-3 * DOCS * OPS
    assert line["detail"]["bad_docs"] == 0
    # the reduced digest equals one process's digest over all documents
    sys.path.insert(0, ROOT)
    from fluidframework_amd import shard
    from fluidframework_amd.synth import make_cfg, tables
    from oracle.oracle import generate
    _, hashes, _ = generate(make_cfg(DOCS, OPS, writers=4, max_lag=8), tables(writers=4), 0, DOCS, threads=2)
    assert line["detail"]["digest"] == f"{shard.digest(hashes):016x}"


def _expected_digest():
    sys.path.insert(0, ROOT)
    from fluidframework_amd import shard
    from fluidframework_amd.synth import make_cfg, tables
    from oracle.oracle import generate
    _, hashes, _ = generate(make_cfg(DOCS, OPS, writers=4, max_lag=8), tables(writers=4), 0, DOCS, threads=2)
    return f"{shard.digest(hashes):016x}"


def _bench_cmd(gpus):
    return [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--docs", str(DOCS), "--ops",
            str(OPS), "--writers", "4", "--max-lag", "8", "--steps", "3", "--warmup", "1", "--dist-backend", "gloo",
            "--traffic-file", "/nonexistent", "--e2e-steps", "0", "--rank-sample-docs", "2"]


def _stub_env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(MTR_BENCH_STUB_ENGINE="bench_stub:StubEngine", OMP_NUM_THREADS="2", **kw)
    return env


def test_bench_gpus_flag_launches_ranks_itself():
    """`bench.py --gpus 2` with no torch.distributed.run around it starts the two ranks itself (VERDICT r05 Next #1):
    the line reports both ranks, the world size the process group saw, both ranks' oracle samples summed, and the
    digest over every document."""
    r = subprocess.run(_bench_cmd(2), env=_stub_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # only rank 0 prints
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["rccl_world_size"] == 2 and line["launcher"] == "bench.py"
    assert line["engine"] == "stub"
    assert line["config"]["docs_total"] == DOCS and line["config"]["docs_per_gpu"] == 3
    assert abs(line["value"] * line["ms_per_step"] / 1000.0 - DOCS * OPS) < 1e-3 * DOCS * OPS
    be = line["bit_exact_sample"]
    assert be["ranks"] == 2 and be["checked_docs"] == 4 and be["equal"] == 4 and be["oracle_errors"] == 0
    assert line["cpu_baseline"] is None  # (rank 0 at N=1 only)
    assert line["detail"]["digest"] == _expected_digest()


def test_bench_rank_sample_mismatch_fails_the_run():
    """A rank whose summaries differ from the oracle's makes the whole run exit non-zero."""
    r = subprocess.run(_bench_cmd(2), env=_stub_env(BENCH_STUB_CORRUPT_RANK="1"), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode != 0
    assert "differ from the CPU oracle" in r.stderr


def test_bench_refuses_world_size_other_than_gpus():
    """Under a launcher that started 1 rank, `--gpus 2` is refused rather than reported as a 2-GPU run."""
    env = _stub_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run(_bench_cmd(2), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "refusing" in r.stderr
