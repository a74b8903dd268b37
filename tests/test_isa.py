"""Static checks of the built libmfhip.so's gfx950 machine code (CPU only, no GPU).

tools/isa_check.py extracts every gfx950 code object from the library, disassembles it and walks
each kernel's control-flow graph:

* no store of more than 64 bits has its data VGPRs overwritten by a VALU within two wait states
  (the gfx950 store-data hazard behind the round-4 k = 256 lean-path nondeterminism, which LLVM
  does not pad when the store's offset is an SGPR; profiles/r05_store_data_hazard.txt);
* every progress / ticket word of the persistent sweeps is stored only after the row stores it
  publishes have landed: the hand-counted `s_waitcnt vmcnt(N)` in front of it must cover them on
  every path of the BUILT code (k_sweep_pair_sys: every earlier store; k_det_sweep2 and the f64
  k_online_sweep and the split sweep k_det_sweep_split (DSGD and online instances), which publish a ticket one or two entries late: every store older than the
  previous ticket store).

A fixture library (tests/isa_fixtures.hip) with one known-bad and one known-good instance of
each pattern shows that the checker finds what it is meant to find.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import isa_check as ic  # noqa: E402

LIB = os.path.join(ROOT, "large-scale-recommendation_amd", "lib", "libmfhip.so")
HIPCC = "/opt/rocm/bin/hipcc"

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(ic.LLVM, "llvm-objdump")),
                                reason="llvm-objdump (ROCm) not installed")


@pytest.fixture(scope="module")
def kern():
    return ic.kernels(LIB)


@pytest.fixture(scope="module")
def fixtures(tmp_path_factory):
    if not shutil.which(HIPCC) and not os.path.exists(HIPCC):
        pytest.skip("hipcc not installed")
    out = str(tmp_path_factory.mktemp("isa") / "fixtures.so")
    subprocess.run([HIPCC, "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out,
                    os.path.join(ROOT, "tests", "isa_fixtures.hip")], check=True, capture_output=True)
    return ic.kernels(out)


def _one(kern, part):
    names = [n for n in kern if part in n]
    assert len(names) == 1, (part, names)
    return {names[0]: kern[names[0]]}


def test_library_holds_the_sweep_kernels(kern):
    for part in ("k_sweep_pair_sys", "k_det_sweep2", "k_det_sweep_splitILi2ELi0E", "k_det_sweep_splitILi2ELi1E", "k_online_sweep",
                 "k_sweep_pair", "k_predict"):
        assert any(part in n for n in kern), part


def test_checker_finds_the_store_data_hazard(fixtures):
    assert ic.store_hazards(_one(fixtures, "k_fixture_bad_store"), ws=2)
    assert not ic.store_hazards(_one(fixtures, "k_fixture_good_store"), ws=2)


def test_checker_finds_an_early_flag_store(fixtures):
    bad, n = ic.flag_store_violations(_one(fixtures, "k_fixture_bad_handoff"), "handoff", ic.progress_flag, "all")
    assert n == 1 and len(bad) == 1
    good, n = ic.flag_store_violations(_one(fixtures, "k_fixture_good_handoff"), "handoff", ic.progress_flag, "all")
    assert n == 1 and not good


def test_no_store_data_hazard_in_the_library(kern):
    bad = ic.store_hazards(kern, ws=2)
    assert not bad, bad[:5]


@pytest.mark.parametrize("kernel_re,mode,flag", ic.CHECKS)
def test_flag_stores_wait_for_the_rows_they_publish(kern, kernel_re, mode, flag):
    bad, n = ic.flag_store_violations(kern, kernel_re, flag, mode)
    assert n > 0, f"no flag store found in {kernel_re}"
    assert not bad, bad[:5]
