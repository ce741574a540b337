"""pytest configuration: the `gpu` marker, import paths, shared fixtures."""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "jpeg-encoder-decoder_amd")
for p in (os.path.join(REPO, "tests"), os.path.join(REPO, "oracle"), PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(REPO, "tests", "golden", "manifest.json")) as f:
        return json.load(f)["cases"]
