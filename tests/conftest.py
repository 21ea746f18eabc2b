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


# Positions with more than 64 legal moves (the oracle's lists, duplicates from promotion
# multiplicity included): move generation then scans and ranks more codes than a wave has lanes
# and k_select's PUCT argmax holds several children per lane (tests/test_oracle_golden.py pins
# the counts)
LONG_LIST_FENS = [
    '1k3/P1PPP/Q3Q/2Q2/Q3Q/R3K w 0 1',       # 72 moves, 54 distinct codes
    '2k2/PP1PP/Q3Q/2Q2/Q3Q/1R2K w 0 1',      # 73, 55
    'k1Q2/3QQ/1Q3/5/1QR1K/R3Q w 0 1',        # 70, all distinct
    'r3k/q3q/2q2/q3q/p1ppp/1K3 b 0 1',       # the first, colours and ranks mirrored
]
