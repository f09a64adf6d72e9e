import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


import pytest  # noqa: E402


@pytest.fixture
def say(capsys):
    """Progress lines for long GPU tests, written past pytest's capture so a runner that
    watches the output sees the test is alive."""

    def _say(msg):
        with capsys.disabled():
            print(msg, flush=True)

    return _say
