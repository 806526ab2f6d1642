import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-sfm-revisited_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsfm_hip.so on the device)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(autouse=True)
def _tuning_isolated(request):
    """Every GPU test runs on the library's tuning state as the session found
    it and leaves it so: every knob (sfm_tune_key's list) is snapshotted before
    the test and restored after it, so a test that switches a scorer or a
    launch shape cannot leak that choice into the tests after it (round 4 ran
    the C2 and band-edge parity tests on k_score_mf after one did)."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    from sfm_amd import _lib
    try:
        snap = _lib.tune_snapshot()
    except _lib.SfmError:
        snap = None
    yield
    if snap is not None:
        _lib.tune_restore(snap)


@pytest.fixture(scope="session", autouse=True)
def _build_oracle():
    # the oracle is test infrastructure: build it if the .so is missing
    lib = os.path.join(ROOT, "oracle", "liboracle_ransac.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"], check=True)
    yield


@pytest.hookimpl(trylast=True)
def pytest_collection_modifyitems(session, config, items):
    """The two-rank GPU test (test_gpu_dist.py) needs its ranks started as
    fresh processes before this process touches the GPU: start them here,
    after collection and deselection, before any test runs.
    torch.cuda.device_count() does not initialise the GPU."""
    if not any("test_gpu_dist.py" in it.nodeid for it in items):
        return
    import tempfile
    import torch
    if torch.cuda.device_count() < 1:
        return
    out = tempfile.mkdtemp(prefix="sfm_dist_")
    port = _free_port()
    procs, logs = [], []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SFM_DIST_OUT=out)
        log = open(os.path.join(out, f"rank{r}.log"), "w")
        logs.append(log)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "helpers", "dist_gpu_worker.py")],
                                      env=env, stdout=log, stderr=subprocess.STDOUT))
    for log in logs:          # the children hold their own descriptors
        log.close()
    config._sfm_dist_ranks = (procs, out)


def _stop_ranks(procs):
    for p in procs:
        if p.poll() is None:
            p.kill()
    for p in procs:
        try:
            p.wait(timeout=30)
        except Exception:
            pass


def pytest_sessionfinish(session, exitstatus):
    """The dist ranks never outlive the session, whether or not their test ran
    (e.g. an earlier failure under -x)."""
    ranks = getattr(session.config, "_sfm_dist_ranks", None)
    if ranks is not None:
        _stop_ranks(ranks[0])


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="session")
def dist_gpu_ranks(request):
    ranks = getattr(request.config, "_sfm_dist_ranks", None)
    if ranks is None:
        pytest.skip("ranks not started (no GPU, or the test was not collected at session start)")
    yield ranks
    _stop_ranks(ranks[0])


def load_golden(name):
    """npz -> nested dict ("group/key" entries become d[group][key])."""
    z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    out = {}
    for k in z.files:
        if "/" in k:
            g, kk = k.split("/", 1)
            out.setdefault(g, {})[kk] = z[k]
        else:
            out[k] = z[k]
    return out


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)
