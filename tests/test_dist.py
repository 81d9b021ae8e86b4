"""The N > 1 path on CPU: two gloo ranks each solve their own block of the global counter-based
stream (oracle as the per-rank solver) and gather the applied moves to rank 0 with the same helpers
bench.py uses (solvempc_amd.dist).  Rank 0 must hold exactly the single-process result."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from solvempc_amd import dist as mdist
from solvempc_amd import workload

N, PER_RANK, WORLD = 20, 48, 2


def _moves(start, count):
    plant = workload.reference_plant()
    ops = oracle.condense(plant, N)
    X, U = workload.mpc_states(1, start, count)
    q, u = oracle.gradient(ops, X, U), oracle.upper_bound(ops, X, U)
    l = np.full(2 * N, -np.finfo(np.float64).max)
    x, st, _, _ = oracle.batch_solve(ops["P"], ops["A"], np.zeros(N), l, oracle.upper_bound(ops, np.zeros(4), 0.0),
                                     q, u, nthreads=1)
    return U + np.where(st == oracle.SOLVED, x[:, 0], 0.0)  # U += x0 (ModelPredictiveControlAPI.cpp:105)


def _worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    r, w, _ = mdist.world_from_env()
    dist.init_process_group("gloo", rank=r, world_size=w)
    start, count = mdist.weak_block(PER_RANK, r)
    moves = torch.from_numpy(_moves(start, count))
    got = mdist.gather_moves(dist, moves, w, r)
    if r == 0:
        out.put(torch.cat(got).numpy())
    dist.barrier()
    dist.destroy_process_group()


def _plant_moves(start, count):
    """BASELINE config 3 for global plants start .. start+count-1: each plant's ctor + one controllerStep
    (oracle.plants_step, the per-rank solver here), the applied U."""
    plant = workload.reference_plant()
    Ad, Bd = workload.randomized_plants(plant, 2, start, count)
    X, U = workload.mpc_states(2, start, count)
    return oracle.plants_step(plant, Ad, Bd, X, U, N, nthreads=1)[0]


def _strong_worker(rank, port, out, total):
    """One rank of the cfg3_strong job: its strong block, padded to the longest block, gathered, trimmed."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    r, w, _ = mdist.world_from_env()
    dist.init_process_group("gloo", rank=r, world_size=w)
    start, count = mdist.strong_block(total, r, w)
    pad = -(-total // w)
    moves = torch.zeros(pad, dtype=torch.float64)
    moves[:count] = torch.from_numpy(_plant_moves(start, count))
    got = mdist.gather_moves(dist, moves, w, r)
    if r == 0:
        out.put(mdist.unpad(got, total, w).numpy())
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gather_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(res, _moves(0, PER_RANK * WORLD))


def test_strong_config3_gather_equals_single_process():
    """bench.py's cfg3_strong job on 2 gloo ranks: ONE global batch of randomised plants (an odd count, so the
    blocks differ by one and the gather pads), each rank solving its block; rank 0's gathered U, trimmed
    (dist.unpad), equals the single-process result for the whole batch."""
    total = 67
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_strong_worker, args=(r, port, q, total)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(res, _plant_moves(0, total))


def test_blocks_tile_the_stream():
    assert [mdist.strong_block(10, r, 3) for r in range(3)] == [(0, 4), (4, 3), (7, 3)]
    assert mdist.weak_block(65536, 3) == (196608, 65536)
    # counter-based states are shard-invariant
    a = np.concatenate([workload.mpc_states(1, s, c)[0] for s, c in (mdist.strong_block(100, r, 4) for r in range(4))])
    np.testing.assert_array_equal(a, workload.mpc_states(1, 0, 100)[0])


def test_bench_launches_its_own_ranks():
    """`python bench.py --gpus 2` spawns its two ranks itself (RANK / WORLD_SIZE / MASTER_* per child,
    before any device call); the dry run does the rendezvous and the per-step gather over gloo and
    rank 0 prints the one JSON line with the world size the gather saw."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--backend", "gloo", "--dry-run",
                        "--steps", "3", "--warmup", "1", "--batch", "1000", "--cfg3-global-batch", "1001"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["dry_run"] is True
    assert rec["collective"] == {"backend": "gloo", "world_size": 2, "gathered": 2000, "matches_stream": True}
    assert rec["scaling"] == "weak"
    # the same line carries BASELINE config 3 as written: one global batch split over the two ranks
    c3 = rec["cfg3_strong"]
    assert c3["scaling"] == "strong" and c3["n_gpus"] == 2 and c3["config"]["global_batch"] == 1001
    assert c3["collective"] == {"backend": "gloo", "world_size": 2, "gathered": 1001, "matches_stream": True}


def test_bench_strong_scaling_splits_one_global_batch():
    """BASELINE config 3 as written: `--workload perplant --scaling strong` splits ONE global batch
    (here 1,001 plants, not a multiple of the world size) into contiguous blocks (dist.strong_block);
    the gather pads every block to the longest and rank 0 recovers exactly the global stream."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--backend", "gloo", "--dry-run",
                        "--workload", "perplant", "--scaling", "strong", "--global-batch", "1001",
                        "--steps", "2", "--warmup", "1"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["scaling"] == "strong" and rec["config"]["global_batch"] == 1001
    assert rec["config"]["batch_per_gpu"] == 501  # rank 0's block
    assert rec["collective"]["gathered"] == 1001 and rec["collective"]["matches_stream"] is True
    assert 1 << 20 == __import__("bench").parse(["--workload", "perplant", "--scaling", "strong"]).global_batch


def test_bench_under_torch_distributed_run():
    """The driver's launcher: `python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr
    127.0.0.1 --master-port P bench.py --gpus 2 ...` (the ranks come from the launcher, bench.py spawns
    none); four steps of the overlapped per-step gather over gloo reach rank 0 intact."""
    import json
    import socket
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(root / "bench.py"),
                        "--gpus", "2", "--backend", "gloo", "--dry-run", "--steps", "4", "--warmup", "2",
                        "--batch", "777"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 4 and rec["warmup"] == 2
    assert rec["collective"] == {"backend": "gloo", "world_size": 2, "gathered": 1554, "matches_stream": True}


def test_bench_parse_seed_per_workload_and_scaling():
    """SURVEY §8d seeds: config 2 seed 1, config 3 (perplant) seed 2, config 4 (quadrotor) seed 3, config 5
    (stream) seed 4, whatever the scaling mode; an explicit --seed always wins."""
    parse = __import__("bench").parse
    want = {"cfg2": 1, "perplant": 2, "quadrotor": 3, "stream": 4}
    for wl, seed in want.items():
        for sc in ("weak", "strong"):
            assert parse(["--workload", wl, "--scaling", sc]).seed == seed, (wl, sc)
            assert parse(["--workload", wl, "--scaling", sc, "--seed", "7"]).seed == 7, (wl, sc)
