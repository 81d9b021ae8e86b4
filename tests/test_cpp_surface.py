"""CPU tests of the C++ drop-in surface (no device needed):

* ``ModelPredictiveControlAPI::from_json`` (solvempc_amd/cpp) against the reference's shape rules and
  error behaviour (src/ModelPredictiveControlAPI.cpp:418-489: nlohmann::detail::type_error::create(0, "")
  after the reference's stderr line; a non-number element is json's type_error 302), and against the
  Python mirror ``solvempc_amd.mpc.from_json``;
* the osqp-eigen-shaped adapter ``include/OsqpEigen/OsqpEigen.h``: a caller written in the reference's
  Eigen call shapes (tests/cpp/reference_caller.cpp, C++11 with the reference's compile flags,
  CMakeLists.txt:21-24) compiles against it and the caller's Eigen (the reference's vendored Eigen
  3.3.9, read through an include path where this container has it) and, with no gfx950 device,
  fails at initSolver() exactly as osqp-eigen reports a failed setup (solverFlag = false, :64);
* the ``solvempc`` CLI (solver.cpp surface) fails loudly without a device or a readable config.
"""
import json
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

from solvempc_amd import mpc

ROOT = Path(__file__).resolve().parents[1]
CPP = ROOT / "tests" / "cpp"
EIGEN = Path("/root/reference/include")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="module")
def from_json_check():
    if os.environ.get("FROM_JSON_CHECK"):  # the ASan / UBSan build (make sanitize)
        return Path(os.environ["FROM_JSON_CHECK"])
    subprocess.run(["make", "-C", str(CPP), "-s", "build/from_json_check"], check=True)
    return CPP / "build" / "from_json_check"


def _run(exe, doc, rows, cols):
    r = subprocess.run([str(exe), json.dumps(doc), str(rows), str(cols)], capture_output=True, text=True, timeout=30)
    assert r.returncode == 0
    return r.stdout.strip(), r.stderr.strip()


OK_CASES = [
    ([5.0], 1, 1, [[5.0]]),                       # RD given as a bare vector (config/MPC_API.json)
    (2.0, 1, 1, [[2.0]]),                         # scalar
    ([1, 2, 3, 4], 4, 1, [[1], [2], [3], [4]]),   # column vector
    ([1, 2, 3, 4], 1, 4, [[1, 2, 3, 4]]),         # row vector
    ([[1, 2], [3, 4]], 2, 2, [[1, 2], [3, 4]]),   # matrix
    ([[-50.0, -150.0, 5500.0, 350.0]], 1, 4, [[-50.0, -150.0, 5500.0, 350.0]]),  # K
    ([], 2, 3, np.zeros((2, 3))),                 # empty array: the requested shape, unset (zeros here)
]
ERR_CASES = [  # (document, rows, cols, reference stderr line or "")
    ([[1, 2], [3]], 2, 2, "Unconsistent matrix size: some rows have different number of columns."),
    ([1, 2, 3], 4, 1, "Expected matrix of size 4x1, received matrix of size 3x1."),
    ([[1, 2, 3]], 2, 3, "Expected matrix of size 2x3, received matrix of size 1x3."),
    ([1, 2, 3], 2, 2, "Expected a matrix, received a vector."),
    ("x", 1, 1, ""),
    (None, 1, 1, ""),
    (True, 1, 1, ""),
    ({"a": 1}, 1, 1, ""),
]


@pytest.mark.parametrize("doc,rows,cols,want", OK_CASES)
def test_from_json_shapes(from_json_check, doc, rows, cols, want):
    out, err = _run(from_json_check, doc, rows, cols)
    f = out.split()
    assert f[0] == "ok", out
    got = np.array([float(v) for v in f[3:]]).reshape(int(f[1]), int(f[2]))
    np.testing.assert_array_equal(got, np.asarray(want, dtype=float))
    np.testing.assert_array_equal(mpc.from_json(doc, rows, cols), got)  # the Python mirror agrees


@pytest.mark.parametrize("doc,rows,cols,line", ERR_CASES)
def test_from_json_errors(from_json_check, doc, rows, cols, line):
    out, err = _run(from_json_check, doc, rows, cols)
    assert out == "type_error 0 [json.exception.type_error.0]", out  # type_error::create(0, "")
    assert err == line
    with pytest.raises(mpc.JsonTypeError):
        mpc.from_json(doc, rows, cols)


def test_from_json_non_number_element(from_json_check):
    out, _ = _run(from_json_check, [[1, "a"]], 1, 2)
    assert out.startswith("type_error 302 "), out  # json's get<double>() of a string


@pytest.mark.skipif(not (EIGEN / "Eigen" / "Dense").exists(), reason="needs an Eigen include directory")
def test_reference_shaped_caller_compiles_against_adapter(tmp_path):
    r = subprocess.run(["make", "-C", str(CPP), "-s", "build/reference_caller", f"EIGEN_INC={EIGEN}"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    if _has_gpu():
        return
    import oracle
    from solvempc_amd import workload

    ops = oracle.condense(workload.reference_plant(), 15)
    f = tmp_path / "in.txt"
    f.write_text("1\n" + "\n".join(" ".join(f"{v:.17g}" for v in ops[k].ravel())
                                   for k in ("P", "A", "Fx", "Fu", "Fr", "Sbar", "Ku", "W0")) + "\n0 0\n0.1 0 0 0\n")
    r = subprocess.run([str(CPP / "build" / "reference_caller"), str(f)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 3 and r.stdout.startswith("initSolver failed"), (r.returncode, r.stdout)


def test_cli_missing_config_is_a_parse_error(tmp_path):
    exe = ROOT / "solvempc_amd" / "solvempc"
    r = subprocess.run([str(exe), "-c", str(tmp_path / "absent.json")], input="", capture_output=True, text=True,
                       timeout=60)
    assert r.returncode != 0
    assert "json.exception.parse_error.101" in r.stderr


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a host with a GPU driver: the device path runs")
def test_cli_without_device_takes_the_solver_flag_exit():
    """BASELINE config 1 on a host with no device: the drop-in's constructor, whose
    condensing runs on the device, reports the failure and leaves solverFlag false, so the CLI takes the
    reference's own exit (`if(!mpc.solverFlag){return 1;}`, solver.cpp:28) instead of aborting."""
    exe = ROOT / "solvempc_amd" / "solvempc"
    r = subprocess.run([str(exe), "-c", str(ROOT / "tests" / "golden" / "plant_mpc_api.json")], input="",
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1, (r.returncode, r.stderr)
    assert "condensing failed" in r.stderr
    assert "Entering control loop" not in r.stdout
