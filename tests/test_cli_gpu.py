"""The reference's own control loop through the MI355X path, on the GPU:

* the ``solvempc`` CLI (src/solver.cpp:13-80 with the serial port replaced by a replay of the same wire
  format, SerialPort.cpp:106-166) run as ``-v -c <config> -N 15 -i <messages> -o <wire>``: every output
  line is the 8-character ``std::to_string(U)`` prefix writePort sends, valid messages (> 30 bytes)
  run ``controllerStep`` and short reads resend the last U (solver.cpp:69-73).  Compared with the
  oracle's controllerStep sequence on the same float-parsed states; the ``-v`` log carries the
  reference's matrix dumps (ModelPredictiveControlAPI.cpp:118-321), checked against the oracle's
  condensed operators at the printed precision;
* the reference-shaped Eigen caller (tests/cpp/reference_caller.cpp over include/OsqpEigen/OsqpEigen.h,
  built in the build container where an Eigen include directory exists) when its binary is present.
"""
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle
from solvempc_amd import workload

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
CFG = ROOT / "tests" / "golden" / "plant_mpc_api.json"
N = 15
LMIN = -np.finfo(np.float64).max


def _messages(k, seed=17):
    """Replay lines: 'dt x0 x1 x2 x3' in the Arduino's %.6f format, every 4th one a short (bad) read."""
    X, _ = workload.mpc_states(seed, 0, k)
    X = X * 0.2
    lines = []
    for i in range(k):
        if i % 4 == 3:
            lines.append("0.01 0.1")  # <= 30 bytes: a bad read (SerialPort.cpp:148)
        else:
            lines.append("0.010000 " + " ".join(f"{v:.6f}" for v in X[i]))
    return lines


def _oracle_wire(lines, plant):
    ops = oracle.condense(plant, N)
    xref = plant["xref"]
    l = np.full(2 * N, LMIN)
    r = oracle.Solver(ops["P"], oracle.gradient(ops, np.zeros(4), 0.0, xref), ops["A"], l,
                      oracle.upper_bound(ops, np.zeros(4), 0.0))
    U, out, iters = 0.0, [], []
    for line in lines:
        if len(line) + 1 > 30:  # readPort: num_bytes > 30
            tok = line.split()
            X = np.array([np.float32(float(t)) for t in tok[1:5]], dtype=np.float64)  # float ref[5]
            assert r.update_gradient(oracle.gradient(ops, X, U, xref))
            assert r.update_upper_bound(oracle.upper_bound(ops, X, U))
            assert r.solve() == oracle.SOLVED
            U += r.x()[0]
            iters.append(r.info().iter)
        out.append(("%f" % U)[:8])  # std::to_string(U), first sizeof(char*) bytes
    _oracle_wire.iters = iters
    return out


def test_cli_replay_matches_oracle_controller(tmp_path, plant):
    lines = _messages(40)
    (tmp_path / "msgs.txt").write_text("\n".join(lines) + "\n")
    wire = tmp_path / "wire.txt"
    r = subprocess.run([str(ROOT / "solvempc_amd" / "solvempc"), "-v", "-c", str(CFG), "-N", str(N),
                        "-i", str(tmp_path / "msgs.txt"), "-o", str(wire)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    got = wire.read_text().split("\n")[:-1]
    want = _oracle_wire(lines, plant)
    assert len(got) == len(lines)
    assert got == want
    log = r.stdout
    assert "[solveMPC]\tVerbose output on." in log and "[MPC API]\tAll QP matrices built successfully." in log
    assert log.count("[solveMPC]\tControl output:") == sum(len(x) + 1 > 30 for x in lines)
    # -v dump of the Hessian (setH :265-270) at the stream's default precision (6 significant digits)
    m = re.search(r"H rows: 15\tH cols: 15\nH:\n((?:.*\n){15})", log)
    assert m, "H dump missing"
    H = np.array([[float(v) for v in row.split()] for row in m.group(1).strip().split("\n")])
    P = oracle.condense(plant, N)["P"]
    np.testing.assert_allclose(H, P, rtol=1e-5, atol=1e-9)
    for name in ("Ad", "Bd", "Sx", "Su", "Sbar", "LL", "Fu", "Fr", "Fx", "Gbar", "Qbar"):
        assert f"\n{name}:\n" in log, name
    # -v also turns on the solver's own output (ModelPredictiveControlAPI.cpp:51 setVerbosity): the
    # setup header once, then per controllerStep the final iterate's summary line and the status block,
    # whose iteration counts are the oracle's
    assert log.count("libmpcq: batched OSQP-v0.6 ADMM on gfx950") == 1
    assert "eps_abs = 1.0e-03, eps_rel = 1.0e-03," in log and "warm start: on, polish: off" in log
    steps = sum(len(x) + 1 > 30 for x in lines)
    assert log.count("status:               solved\n") == steps
    its = [int(v) for v in re.findall(r"number of iterations: (\d+)", log)]
    assert its == _oracle_wire.iters
    rows = re.findall(r"iter   objective    pri res    dua res    rho        time\n(.*)\n", log)
    assert len(rows) == steps
    for row, want in zip(rows, _oracle_wire.iters):
        it, obj, pri, dua, rho, t = row.split()
        assert int(it) == want and np.isfinite(float(obj)) and float(pri) >= 0 and float(dua) >= 0
        assert float(rho) > 0 and t.endswith("s")


def test_reference_shaped_eigen_caller_on_device(tmp_path, plant):
    exe = ROOT / "tests" / "cpp" / "build" / "reference_caller"
    if not exe.exists():
        pytest.skip("reference_caller is built where an Eigen include directory exists (build())")
    ops = oracle.condense(plant, N)
    X, _ = workload.mpc_states(5, 0, 12)
    X = X * 0.2  # the reference's ctor starts from X = 0, U = 0 (:22-23); the caller does too
    f = tmp_path / "in.txt"
    f.write_text(f"{len(X)}\n" + "\n".join(" ".join(f"{v:.17g}" for v in ops[k].ravel())
                                           for k in ("P", "A", "Fx", "Fu", "Fr", "Sbar", "Ku", "W0"))
 + "\n0 0\n" + "\n".join(" ".join(f"{v:.17g}" for v in x) for x in X) + "\n")
    r = subprocess.run([str(exe), str(f)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.array([[float(v) for v in line.split()] for line in r.stdout.strip().split("\n")])
    l = np.full(2 * N, LMIN)
    ref = oracle.Solver(ops["P"], np.zeros(N), ops["A"], l, oracle.upper_bound(ops, np.zeros(4), 0.0))
    U = 0.0
    for k, x in enumerate(X):
        assert ref.update_gradient(oracle.gradient(ops, x, U)) and ref.update_upper_bound(oracle.upper_bound(ops, x, U))
        assert ref.solve() == oracle.SOLVED
        U += ref.x()[0]
        assert abs(got[k, 0] - U) < 1e-9 and got[k, 1] == 1 and got[k, 2] == ref.info().iter, (k, got[k], U)
