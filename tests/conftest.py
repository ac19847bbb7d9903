import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, 'tests', 'golden')
sys.path.insert(0, os.path.join(REPO, 'tests'))
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs on the GPU box)')
    config.addinivalue_line('markers', 'slow: long-running test')


@pytest.fixture(scope='session')
def golden():
    return GOLDEN


@pytest.fixture(scope='session')
def tmpdir_session(tmp_path_factory):
    return tmp_path_factory.mktemp('rwkv')
