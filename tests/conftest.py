import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (run with -m gpu on the GPU box)')
    config.addinivalue_line('markers', 'slow: longer CPU test')


def load_golden(name):
    import json
    with open(os.path.join(GOLDEN, name + '.json')) as fh:
        return json.load(fh)


@pytest.fixture(scope='session')
def golden():
    return load_golden
