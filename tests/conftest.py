import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(Path(__file__).resolve().parent))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsamplers_hip.so)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture
def parity_record(request):
    """record(metric, value, bound, **extra): one JSON line per measured parity error, appended to
    ``$SAMPLERS_AMD_PARITY_LOG`` (default ``gpurun_out/parity_record.jsonl`` under the repo root,
    which gpurun merges back), and attached to the test report (``record_property``), so the
    margin to each bound is on record and not only pass / fail."""
    import json
    import time

    path = Path(os.environ.get("SAMPLERS_AMD_PARITY_LOG", ROOT / "gpurun_out" / "parity_record.jsonl"))

    def record(metric: str, value: float, bound: float | None = None, **extra) -> None:
        rec = {"test": request.node.nodeid, "metric": metric, "value": float(value),
               "bound": bound, "margin": None if not bound else float(value) / bound,
               "time": time.strftime("%Y-%m-%dT%H:%M:%S"), **extra}
        request.node.user_properties.append((metric, float(value)))
        try:
            path.parent.mkdir(parents=True, exist_ok=True)
            with open(path, "a") as f:
                f.write(json.dumps(rec) + "\n")
        except OSError:
            pass

    return record
