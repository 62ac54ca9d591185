"""ASan + UBSan build of the host C++ feeder builder (csrc/pgw_feeder.cpp;
SURVEY section 5): tests/c/feeder_sanitize.cpp is compiled with it under
-fsanitize=address,undefined, given the element lists of the shipped IEEE-13
feeder and the two test feeders, and must reproduce the library's Y, Z,
source currents, no-load voltages and load-element reduction (to the last
bits), then
reject malformed input cleanly.  CPU only (g++)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from powergridworld_amd import _lib
from powergridworld_amd.distribution_system.feeder import Feeder, load_feeder_spec

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "powergridworld_amd", "csrc")
FEEDERS = ["IEEE13Nodeckt.dss", os.path.join(REPO, "tests", "data", "regcap_feeder.dss"),
           os.path.join(REPO, "tests", "data", "feeder48.dss"),
           os.path.join(REPO, "tests", "data", "xfmr3_feeder.dss")]


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("asan") / "feeder_sanitize")
    subprocess.run(["g++", "-std=c++17", "-O2", "-g", "-fno-omit-frame-pointer", "-ffp-contract=off",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                    "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "c", "feeder_sanitize.cpp"), os.path.join(CSRC, "pgw_feeder.cpp"),
                    "-o", out], check=True)
    return out


@pytest.mark.parametrize("feeder_file", FEEDERS, ids=["ieee13", "regcap", "feeder48", "xfmr3"])
def test_feeder_builder_under_asan_ubsan(driver, feeder_file):
    f = Feeder(load_feeder_spec(feeder_file))
    els = f.elements()
    arr = (_lib.FeederElem * len(els))(*els)
    n, m = f.n, f.m
    out_nodes = np.arange(n, dtype=np.int32)
    blob = (np.array([len(els), n, m, n], np.int32).tobytes() + bytes(arr) + f.elem_p.astype(np.int32).tobytes()
            + f.elem_q.astype(np.int32).tobytes() + out_nodes.tobytes())
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([driver], input=blob, capture_output=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr.decode()[-4000:]
    got = np.frombuffer(r.stdout, np.float64)
    sizes = [2 * n * n, 2 * n * n, 2 * n, 2 * n, 2 * m * m, 2 * m, 2 * n * m, 2 * n]
    assert got.size == sum(sizes)
    parts = np.split(got, np.cumsum(sizes)[:-1])
    W, U0, G, V0o = f.reduce_rows(out_nodes)
    want = [f.Y, f.Z, f.I_src, f.V0, W, U0, G, V0o]
    # the instrumented build rounds a few complex products / divisions
    # differently in the last bit (std::complex codegen under the sanitizers)
    for g, w in zip(parts, want):
        w = np.ascontiguousarray(w).view(np.float64).ravel()
        np.testing.assert_allclose(g, w, rtol=1e-12, atol=1e-12 * max(np.abs(w).max(), 1e-300))
