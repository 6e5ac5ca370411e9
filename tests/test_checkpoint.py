"""Checkpoint file handling without a GPU: the .chk layout (id 3252359,
SampleCollector.f90:76, written through .chk_tmp and a rename, :174-187),
rejection of foreign files and configurations, and the chain-file cut-back
that makes a resumed run's files continue seamlessly."""
import struct

import numpy as np
import pytest

from cosmomc_amd.chains import ChainWriter
from cosmomc_amd.checkpoint import CHK_ID, read_checkpoint, write_checkpoint


class FakeSampler:
    """Duck-typed stand-in for BatchedMCMC's state calls (host only)."""

    def __init__(self, W=4, np_=3, used=(1, 2), hist_cap=0):
        self.W, self.np, self.params_used = W, np_, list(used)
        self._hist_cap = hist_cap
        self.image = bytes(range(37))
        self.loaded = None
        self.cov = None
        self.hist = np.arange(5 * (len(used) + 1) * W, dtype=np.float64).reshape(5, len(used) + 1, W)
        self.restored = None

    def save_state(self):
        return self.image

    def load_state(self, image):
        self.loaded = image

    def set_covariance(self, cov):
        self.cov = cov

    def history_count(self):
        return len(self.hist)

    def history_host(self, first, count):
        return self.hist[first:first + count]

    def history_restore(self, first, rows, terms=None):
        self.restored = (first, np.array(rows))


def test_roundtrip_and_layout(tmp_path):
    root = str(tmp_path / "x")
    s = FakeSampler(hist_cap=3)
    cov = np.array([[1.0, 0.1], [0.1, 2.0]])
    path = write_checkpoint(root, s, cov, collector={"num_sample": 7, "MaxLike": 12.5})
    raw = open(path, "rb").read()
    assert struct.unpack_from("<i", raw, 0)[0] == CHK_ID
    assert not (tmp_path / "x.chk_tmp").exists()
    t = FakeSampler(hist_cap=3)
    assert read_checkpoint(root, t) == {"num_sample": 7, "MaxLike": 12.5}
    assert t.loaded == s.image
    np.testing.assert_array_equal(t.cov, cov)
    first, rows = t.restored
    assert first == 2                                     # the ring kept the last 3 of 5 rows
    np.testing.assert_array_equal(rows, s.hist[2:])


def test_rejects_foreign_file_and_other_config(tmp_path):
    root = str(tmp_path / "bad")
    with open(root + ".chk", "wb") as f:
        f.write(struct.pack("<ii", 1234, 1) + b"\0" * 32)
    with pytest.raises(ValueError, match="invalid checkpoint"):
        read_checkpoint(root, FakeSampler())
    write_checkpoint(root, FakeSampler(W=4), np.eye(2))
    with pytest.raises(ValueError, match="different sampler"):
        read_checkpoint(root, FakeSampler(W=8))


def test_chain_files_cut_back_to_checkpoint(tmp_path):
    root = str(tmp_path / "c")
    rows = np.zeros((4, 2, 2))
    rows[:, 0, :] = np.array([[1.0, 5.0], [1.0, 5.0], [2.0, 6.0], [3.0, 6.0]])
    rows[:, 1, :] = 10.0
    cw = ChainWriter(root, ["a"], burn_in=-1)
    cw.add_rows(rows)
    st = cw.checkpoint_state(2)
    before = {w: open(f"{root}_{w + 1}.txt").read() for w in range(2)}
    cw.add_rows(rows + 1.0)                       # rows written after the checkpoint
    cw2 = ChainWriter(root, ["a"], burn_in=-1)
    cw2.restore(st, 2)
    assert {w: open(f"{root}_{w + 1}.txt").read() for w in range(2)} == before
    assert cw2.pending[0][1] == 1 and cw2.pending[1][1] == 2     # open runs carried over
    cw2.add_rows(rows[:1] + 7.0)                  # both walkers move off their open points
    cw2.close()
    c1 = np.loadtxt(f"{root}_2.txt", ndmin=2)
    np.testing.assert_array_equal(c1[:, 0], [2, 2])
