import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    config.addinivalue_line("markers", "two_process: two processes share the one GPU (run last)")


def pytest_collection_modifyitems(config, items):
    # two processes on one GPU are outside the deployment rule (one process per GPU) and their
    # run-to-run determinism is a known open item ("two-process nondeterminism"):
    # run them after every single-process test, so that under -x a failure there cannot hide the rest
    items.sort(key=lambda it: it.get_closest_marker("two_process") is not None)


@pytest.fixture(scope="session")
def unproject_cases():
    data = np.load(os.path.join(GOLDEN, "unproject_cases.npz"))
    with open(os.path.join(GOLDEN, "unproject_cases.json")) as fh:
        meta = json.load(fh)
    out = []
    for m in meta:
        n = m["name"]
        case = dict(m)
        for k in ("image", "depth", "points", "colors", "bounds"):
            case[k] = data[f"{n}__{k}"]
        out.append(case)
    return out


@pytest.fixture(scope="session")
def pipeline_case():
    data = np.load(os.path.join(GOLDEN, "pipeline_case.npz"))
    with open(os.path.join(GOLDEN, "pipeline_case.json")) as fh:
        summary = json.load(fh)
    return {"image": data["image"], "depth": data["depth"], "summary": summary}


@pytest.fixture(scope="session")
def routes_golden():
    with open(os.path.join(GOLDEN, "routes.json")) as fh:
        return json.load(fh)
