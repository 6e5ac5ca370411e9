"""A host stand-in for BatchedMCMC's collector interface (history ring +
cmbs_collector_*), built on the oracle's item-by-item restatement, so that
ChainCollector's cross-rank logic runs on CPU with gloo.  Test helper only."""
import numpy as np

import pyoracle as po


class FakeCollectorSampler:
    """W synthetic chains (global walker ids first_walker ..): each step a
    chain moves (AR(1) step in a random subset of its parameters) with
    probability 0.6, else stays -- deterministic per global walker."""

    def __init__(self, W, n=3, first_walker=0, seed=11):
        self.W, self.n = W, n
        self.params_used = list(range(1, n + 1))
        self.first_walker = first_walker
        self.rngs = [np.random.default_rng([seed, first_walker + w]) for w in range(W)]
        self.cur = np.array([r.standard_normal(n) * 2 for r in self.rngs])
        self.rows = []
        self.states = None

    def step(self, k):
        for _ in range(k):
            for w, r in enumerate(self.rngs):
                if r.random() < 0.6:
                    mask = r.random(self.n) < 0.7
                    self.cur[w] = np.where(mask, 0.5 * self.cur[w] + 0.87 * r.standard_normal(self.n), self.cur[w])
            row = np.concatenate([self.cur.T, 0.5 * (self.cur ** 2).sum(axis=1)[None, :]], axis=0)
            self.rows.append(row)

    def history_count(self):
        return len(self.rows)

    def collector_enable(self, cap):
        self.states = [{"items": [], "sample_num": 0, "burn": False, "changes": None} for _ in range(self.W)]
        self.thin = np.ones(self.W, dtype=int)

    def collector_add(self, steps, min_update, check_burn=True):
        rows = np.array(self.rows)
        for w in range(self.W):
            po.collector_samples(rows[:, :, w], steps, min_update, check_burn, int(self.thin[w]), self.states[w])

    def collector_state(self):
        count = np.array([len(s["items"]) for s in self.states], dtype=np.int32)
        burn = np.array([int(s["burn"]) for s in self.states], dtype=np.int32)
        return np.zeros(self.W, dtype=np.int32), count, burn, self.thin.astype(np.int32)

    def collector_thin(self, limit):
        for w, s in enumerate(self.states):
            if len(s["items"]) > limit:
                s["items"] = s["items"][::2]
                self.thin[w] *= 2

    def _window(self, w):
        it = self.states[w]["items"]
        c = len(it)
        return np.array(self.rows)[it[c // 2 - 1:], :self.n, w]

    def collector_moments(self, gmean=None):
        import torch
        n = self.n
        if gmean is None:
            out = np.zeros(2 + n + 2 * n * n)
        else:
            out = np.zeros(n * n)
            g = np.asarray(gmean.cpu() if hasattr(gmean, "cpu") else gmean)
        for w in range(self.W):
            x = self._window(w)
            cw = x.shape[0]
            m = x.mean(axis=0)
            C = (x - m).T @ (x - m) / cw
            if gmean is None:
                out[0] += cw
                out[1:1 + n] += cw * m
                out[1 + n:1 + n + n * n] += cw * C.ravel()
                out[1 + n + n * n:1 + n + 2 * n * n] += C.ravel()
                out[-1] += 1
            else:
                out += cw * np.outer(m - g, m - g).ravel()
        return torch.tensor(out, dtype=torch.float64)

    def collector_limits(self, params, limfrac):
        import torch
        out = np.zeros((self.W, len(params), 2))
        for w in range(self.W):
            x = self._window(w)
            for c, j in enumerate(params):
                out[w, c] = po.confid_val(x[:, j], limfrac)
        return torch.tensor(out)

    def set_covariance(self, cov):
        pass

    device = "cpu"
