import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def make_locked(*targets, jobs=1, timeout=900):
    """`make <targets>` serialised across pytest-xdist workers per target (a worker must never dlopen
    a fake library another worker is relinking, and two workers must not write the same object).
    One lock per target, taken in sorted order: a long sanitizer build does not hold up the fakes."""
    import contextlib
    import fcntl

    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    with contextlib.ExitStack() as stack:
        for t in sorted(set(targets)):
            lk = stack.enter_context(open(os.path.join(ROOT, "build", f".make-{t}.lock"), "w"))
            fcntl.flock(lk, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-C", ROOT, f"-j{jobs}", *targets], capture_output=True, text=True,
                           timeout=timeout)
    assert r.returncode == 0, r.stderr[-2000:]
    return r


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box with -m gpu)")
    config.addinivalue_line("markers", "slow: takes more than a few seconds")
    # The native core is built in-tree; build it once if this checkout has not been built yet.
    try:
        import gpumon._core  # noqa: F401
    except ImportError:
        subprocess.run(["make", "-C", ROOT, "-j8", "core"], check=True, stdout=subprocess.DEVNULL)


@pytest.fixture
def core():
    from gpumon import core as _c

    return _c()


@pytest.fixture
def mock_exporter(core):
    """Factory for started mock exporters on an ephemeral localhost port; stopped at teardown."""
    made = []

    def make(**over):
        cfg = {"backend": "mock:gpus=2", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0.0,
               "host": "node-a", "http_threads": 1}
        cfg.update(over)
        ex = core.Exporter(cfg)
        ex.start()
        made.append(ex)
        return ex

    yield make
    for ex in made:
        ex.stop()
