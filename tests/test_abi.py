"""The C-ABI library: loads on a CPU-only machine, exports every declared symbol, JVM helpers."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import coracle
import mf_oracle as O
import mfhip
from mfhip import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mfhip.h")
TESTING_HEADER = os.path.join(ROOT, "include", "mfhip_testing.h")


def declared_functions(path=HEADER):
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(mf_\w+)\s*\(", txt, flags=re.M)))


def test_library_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 30
    lib = C.CDLL(L.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(L.EXPORTS) == names
    hooks = declared_functions(TESTING_HEADER)
    for n in hooks:
        assert hasattr(lib, n), n
    assert sorted(L.TESTING_EXPORTS) == hooks
    assert not set(hooks) & set(names)


def test_public_header_is_the_product_surface():
    """include/mfhip.h holds the SURVEY 8b surface plus stats and I/O: no debug hooks, no
    experiment knobs (those live in mfhip_testing.h / environment variables)."""
    names = declared_functions()
    assert not [n for n in names if n.startswith("mf_debug") or "fast_" in n]
    assert "item_split" not in open(HEADER).read()


def test_params_defaults_match_reference():
    p = L.default_params()
    assert p.num_factors == 10 and p.iterations == 10 and p.lambda_ == 1.0   # MatrixFactorization.scala:201-211
    assert p.learning_rate == 0.001 and p.lr_method == 0                     # DSGDforMF.scala:163-169
    assert p.num_blocks == 1 and p.seed == 0 and p.has_seed == 1             # :213-219, getOrElse(1)
    assert p.online_learning_rate == 0.01                                    # SparkExample.scala:33


def test_version_and_device_count():
    assert "gfx950" in mfhip.version()
    assert mfhip.device_count() >= 0


def test_no_silent_cpu_fallback():
    if mfhip.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(mfhip.MFNoDeviceError):
        mfhip.Context(L.default_params())


def test_invalid_params_rejected():
    p = L.default_params()
    p.num_factors = 0
    with pytest.raises(mfhip.MFError):
        mfhip.Context(p)


def test_jvm_helpers_match_oracle():
    for seed in (0, 42, -8, 2**45):
        for n in (0, 1, 5, 333):
            assert mfhip.jvm.shuffle(seed, n).tolist() == coracle.scala_shuffle(seed, n).tolist()
    for id_ in (-3, 0, 9, 2**31 - 1):
        for nb in (1, 4, 7):
            assert mfhip.jvm.block_of(id_, 11, nb) == O.block_of(id_, 11, nb)
    assert np.array_equal(mfhip.jvm.random_factors(5, 7), O.random_factors(7, O.JavaRandom(5)))
    for m, arg in ((0, 0), (1, 0), (2, 2.0), (3, 0.5), (4, 0.5)):
        assert mfhip.jvm.learning_rate(m, 0.01, 3, 0.5, arg) == O.learning_rate(m, 0.01, 3, 0.5, arg)


def test_last_error_is_set():
    lib = L.lib()
    assert lib.mf_jvm_shuffle(0, -1, None) == L.MF_ERR_INVALID
    assert b"bad argument" in lib.mf_last_error()


def test_jni_shim_compiles_against_the_header():
    """jni/mfhip_jni.c (the binding INTEGRATION.md gives a Scala maintainer) against include/mfhip.h:
    every call's arity and pointer types must match the C ABI (-Werror).  No JDK here, so a
    minimal jni.h stand-in (tests/jni_stub) supplies the JNI types; nothing is linked or run."""
    import shutil
    import subprocess
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("no gcc")
    r = subprocess.run([gcc, "-std=c99", "-fsyntax-only", "-Wall", "-Wextra", "-Wno-unused-parameter", "-Werror",
                        "-Werror=incompatible-pointer-types", "-Werror=implicit-function-declaration",
                        "-I", os.path.join(ROOT, "tests", "jni_stub"), "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "jni", "mfhip_jni.c")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_every_java_native_has_a_jni_function():
    java = open(os.path.join(ROOT, "jni", "MfHip.java")).read()
    natives = set(re.findall(r"public static native [\w\[\]]+ (\w+)\(", java))
    shim = open(os.path.join(ROOT, "jni", "mfhip_jni.c")).read()
    defined = set(re.findall(r"JFN\((\w+)\)\(", shim))
    assert natives and natives == defined, (natives ^ defined)
