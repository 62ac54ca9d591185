import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


def golden_path(name):
    return os.path.join(GOLDEN, name + ".npz")


@pytest.fixture(scope="session")
def exo_frame():
    import pandas as pd
    df = pd.read_csv(os.path.join(GOLDEN, "exogenous_synthetic.csv.gz"), index_col=0)
    df.index = pd.DatetimeIndex(df.index)
    return df
