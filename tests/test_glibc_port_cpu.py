"""CPU pin of the device RNG's log / pow (csrc/glibc_math.h).

numpy's legacy gamma sampler calls glibc's log and pow; csrc/glibc_math.h ports their FMA builds
(tables from libm via tools/glibc_tables.py).  A host build of that same header must equal this
machine's glibc bit for bit: tests/glibc_port_check.cpp draws 10^8 arguments per case (4 processes x
2.5 x 10^7), in the gamma loop's ranges (log(1 - U), log((1 - U) / 0.6), pow(U, 1/0.6),
pow(0.4 + 0.6 Y, 1/0.6)) and general ones (positive doubles over the whole range; pow with
x in [2^-200, 2^200], |y| <= 40: subnormal to huge results, exp's special case included)."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
N_PER_PROC, PROCS = 25_000_000, 4


@pytest.fixture(scope='module')
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp('glibc') / 'glibc_port_check')
    subprocess.check_call(['g++', '-O2', '-ffp-contract=off', '-std=c++17', os.path.join(HERE, 'glibc_port_check.cpp'),
                           '-o', exe, '-lm'])
    return exe


def test_tables_are_this_libm():
    """The committed tables equal what tools/glibc_tables.py extracts from the running system's libm
    (skipped on an image with another libm: the bitwise check below then says whether the port
    still holds there)."""
    sys.path.insert(0, os.path.join(REPO, 'tools'))
    import glibc_tables
    hdr = os.path.join(REPO, 'minitchess_alphazero_amd', 'csrc', 'glibc_math_tables.h')
    t, meta = glibc_tables.extract()
    if meta['sha256'] not in open(hdr).read():
        pytest.skip(f'libm {meta["sha256"][:16]} is not the one the tables came from')
    assert glibc_tables.render(t, meta) == open(hdr).read()


def test_port_equals_glibc_1e8(checker):
    procs = [subprocess.Popen([checker, str(N_PER_PROC), str(1000 + i)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for i in range(PROCS)]
    total = {}
    for p in procs:
        out, err = p.communicate(timeout=600)
        res = json.loads(out.strip().splitlines()[-1])
        for k, (bad, n) in res.items():
            b0, n0 = total.get(k, (0, 0))
            total[k] = (b0 + bad, n0 + n)
        assert p.returncode in (0, 1), err
    print(json.dumps(total))
    for k, (bad, n) in total.items():
        assert n >= (PROCS * N_PER_PROC if k != 'log_general' else PROCS * N_PER_PROC // 2), (k, n)
        assert bad == 0, (k, bad, n)
