"""The compare-exchange networks compiled into the kernels are correct
(0-1 principle, exhaustive) and the header is up to date with its generator."""
import itertools
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "etcd_amd", "csrc")
HDR = os.path.join(CSRC, "qb_networks.h")


def parse():
    sel, srt = {}, {}
    for line in open(HDR):
        m = re.match(r"template <> struct (SelNet|SortNet)<(\d+)> \{(.*)\};", line)
        if not m:
            continue
        kind, n, body = m.group(1), int(m.group(2)), m.group(3)
        K = int(re.search(r"K = (\d+)", body).group(1))
        A = [int(x) for x in re.search(r"A\[\d+\] = \{([^}]*)\}", body).group(1).split(",")]
        B = [int(x) for x in re.search(r"B\[\d+\] = \{([^}]*)\}", body).group(1).split(",")]
        net = list(zip(A, B))[:K]
        if kind == "SelNet":
            pos = int(re.search(r"POS = (\d+)", body).group(1))
            sel[n] = (pos, net)
        else:
            srt[n] = net
    return sel, srt


def run(net, v):
    v = list(v)
    for a, b in net:
        if v[b] < v[a]:
            v[a], v[b] = v[b], v[a]
    return v


def test_header_is_current(tmp_path):
    out = tmp_path / "n.h"
    subprocess.check_call([sys.executable, os.path.join(CSRC, "gen_networks.py"), str(out)],
                          stdout=subprocess.DEVNULL)
    assert out.read_text() == open(HDR).read()


@pytest.mark.parametrize("n", range(1, 17))
def test_selection_networks(n):
    sel, _ = parse()
    pos, net = sel[n]
    assert pos == n - (n // 2 + 1)  # majority.go:170
    for bits in itertools.product((0, 1), repeat=n):
        assert run(net, bits)[pos] == sorted(bits)[pos]


@pytest.mark.parametrize("w", range(2, 17))
def test_sorting_networks(w):
    _, srt = parse()
    for bits in itertools.product((0, 1), repeat=w):
        assert run(srt[w], bits) == sorted(bits)
