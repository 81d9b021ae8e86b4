"""Static register / scratch budget of the benched kernels (CPU only: the gfx950 code objects' metadata,
tools/kernel_resources.py).  DESIGN.md states these numbers; rocprofv3's Scratch_Size column of the kernel
traces under profiles/ shows the same on the GPU."""
import os
import shutil

import pytest

import tools.kernel_resources as kr

pytestmark = pytest.mark.skipif(not os.path.isdir(kr.BUILD) or shutil.which("c++filt") is None
                                or not os.path.exists(f"{kr.LLVM}/clang-offload-bundler"),
                                reason="needs the built objects and the ROCm LLVM tools")


@pytest.fixture(scope="module")
def rows():
    return {r["kernel"]: r for r in kr.table()}


def _one(rows, prefix):
    hit = [r for k, r in rows.items() if k.startswith(prefix)]
    assert len(hit) == 1, (prefix, [r["kernel"] for r in hit])
    return hit[0]


def test_config2_tile_kernels_do_not_spill(rows):
    # config 2's mixed headline and its f64 variant: paired loop, 2 waves/SIMD, 256 VGPRs, no scratch
    for mix in ("true", "false"):
        r = _one(rows, f"void mpcq::admm_tile_kernel<double, 5, 10, true, true, 1, 2, true, 4, false, {mix}>")
        assert r["scratch"] == 0 and r["vgpr_spill"] == 0 and r["vgpr"] <= 256


def test_config3_plant_kernel_budget(rows):
    # three plants per wave at 3 waves/SIMD: 168 VGPRs, the spills outside the loop
    r = _one(rows, "void mpcq::plant_step_kernel<double, 20, 3, 3, 4>")
    assert r["vgpr"] <= 168 and r["scratch"] <= 72


def test_config4_mimo_solve_budget(rows):
    r = _one(rows, "void mpcq::mimo_solve_kernel<4, true>")
    assert r["vgpr"] <= 256 and r["scratch"] <= 48
