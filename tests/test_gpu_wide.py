"""GPU parity for WIDE configs (> 16 slots, wave-per-group radix select)."""
import random

import numpy as np
import pytest
import torch

from etcd_amd.quorum import batch
from tests import oracle_c as oc
from tests.test_oracle_c import _random_wide

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _grp(off, vals, flags, max_slots=None):
    dev = torch.device(DEV)
    return batch.WideGroups(torch.from_numpy(off.view(np.int32).copy()).to(dev),
                            batch.from_u64(vals if vals.size else np.zeros(2, np.uint64), dev),
                            torch.from_numpy(flags if flags.size else np.zeros(1, np.uint8)).to(dev),
                            max_slots=max_slots)


@pytest.mark.parametrize("smax,big,seed", [(64, True, 1), (128, False, 2), (256, True, 3),
                                          (512, False, 4), (1024, True, 5), (20, True, 6)])
def test_wide_vs_oracle(smax, big, seed):
    rng = random.Random(seed)
    G = 3000 if smax <= 256 else 600
    off, vals, flags = _random_wide(rng, G, smax, big)
    grp = _grp(off, vals, flags)
    c, v = grp.committed_vote()
    ec, ev = oc.wide_eval(off, vals, flags)
    assert np.array_equal(batch.as_u64(c), ec)
    assert np.array_equal(v.cpu().numpy(), ev)


def test_wide_equals_csr_on_small_groups():
    grp_csr = batch.CsrGroups.synth(0x5EED0004, "joint", 20000, device=DEV)
    off = grp_csr.off.cpu().numpy().view(np.uint32)
    cfg = grp_csr.cfg.cpu().numpy().view(np.uint32)
    votes = grp_csr.votes.cpu().numpy().view(np.uint32)
    flags = np.zeros(int(off[-1]), np.uint8)
    for g in range(len(cfg)):
        for j in range(int(off[g + 1] - off[g])):
            f = ((cfg[g] >> j) & 1) | (((cfg[g] >> (16 + j)) & 1) << 1)
            f |= ((votes[g] >> j) & 1) << 2
            f |= ((votes[g] >> (16 + j)) & 1) << 3
            flags[off[g] + j] = f
    vals = batch.as_u64(grp_csr.match)[: off[-1]]
    grp = _grp(off, vals, flags)
    c, v = grp.committed_vote()
    c2, v2 = grp_csr.committed_vote()
    assert torch.equal(c, c2) and torch.equal(v, v2)


def test_wide_compile_and_empty():
    cw = batch.compile_configs_wide([range(1, 40), [], range(5, 9)], [range(30, 70), [], []],
                                    [[], [1000], [9]])
    vals = np.arange(len(cw.slot_ids), dtype=np.uint64) * 3
    grp = batch.WideGroups.from_compiled(cw, vals, device=DEV)
    c, v = grp.committed_vote()
    ec, ev = oc.wide_eval(cw.off, vals, cw.flags)
    assert np.array_equal(batch.as_u64(c), ec) and np.array_equal(v.cpu().numpy(), ev)
    assert batch.as_u64(c)[1] == (1 << 64) - 1 and v.cpu().numpy()[1] == 3
