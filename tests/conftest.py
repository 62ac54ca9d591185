import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    # multi-process GPU tests fork their ranks from a forkserver started here,
    # before this process touches the GPU: no rank is a fork or an exec of a
    # GPU-initialised process
    mark = (config.option.markexpr or "").strip()
    if mark == "gpu" or (mark and "not gpu" not in mark and "gpu" in mark):
        import multiprocessing.forkserver as fs
        fs.ensure_running()


def golden_path(name):
    return os.path.join(GOLDEN, name + ".npz")


@pytest.fixture(scope="session")
def exo_frame():
    import numpy as np
    import pandas as pd
    with np.load(os.path.join(GOLDEN, "exogenous_synthetic.npz"), allow_pickle=False) as z:
        idx = pd.DatetimeIndex(z["index_ns"].astype("datetime64[ns]"))
        return pd.DataFrame(z["values"], index=idx, columns=[str(c) for c in z["columns"]])
