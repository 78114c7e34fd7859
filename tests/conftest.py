import contextlib
import os
import sys
import threading
import time

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))
GOLDEN = os.path.join(HERE, "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device and libge.so")


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    oracle_lib.build()
    return oracle_lib


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
    return load


@pytest.fixture(scope="session")
def ctx():
    import ge_amd
    c = ge_amd.Context(0)
    yield c
    c.close()


@pytest.fixture
def heartbeat(pytestconfig):
    """Context manager printing a line past pytest's output capture every `every`
    seconds while a long device call runs (the C4/C5 partitions): a GPU run that
    stays silent for minutes is taken for a hung one."""
    capman = pytestconfig.pluginmanager.getplugin("capturemanager")

    @contextlib.contextmanager
    def run(label, every=30.0):
        stop = threading.Event()
        t0 = time.perf_counter()

        def beat():
            while not stop.wait(every):
                msg = f"[{label}: {time.perf_counter() - t0:.0f} s]\n"
                if capman is not None:
                    with capman.global_and_fixture_disabled():
                        sys.stderr.write(msg)
                        sys.stderr.flush()
                else:
                    sys.stderr.write(msg)
                    sys.stderr.flush()

        th = threading.Thread(target=beat, daemon=True)
        th.start()
        try:
            yield
        finally:
            stop.set()
            th.join()
    return run
