"""Checkpoint and resume of a batched run (``root.chk``).

Reference: with ``checkpoint = T`` the collector writes ``rootname.chk``
through ``rootname.chk_tmp`` and a rename (TMpiChainCollector_WriteCheckpoint,
source/SampleCollector.f90:174-187): the id 3252359 (:76), then
TMpiChainCollector_SaveState (:139-151) -- thin factor, burn-in flags,
flukecheck, update frequency, the stored samples -- and the sampler's state
(num_sample, MaxLike, MaxLikeParams, num_accept and the proposal matrix,
MCMC.f90:98-114, 199-218, propose.f90:308-325).  A restart reads the last row
of the chain file for the point and continues with a fresh random sequence
(GeneralSetup.f90:123-131).

Here the file carries the same pieces for every walker plus the complete
device chain state (``cmbs_save_state``: RANMAR tables, proposer cycle and
rotation state), so a resumed run continues each chain exactly -- the chain
files and the convergence test come out as if the run had never stopped.

Layout (little endian): int32 3252359, int32 version, uint64 n, n bytes of
JSON (collector and host state), uint64 m, m bytes of the sampler image,
uint64 h, h bytes of history rows (float64, history_host layout).
"""
from __future__ import annotations

import json
import os
import struct

import numpy as np

CHK_ID = 3252359          # SampleCollector.f90:76
VERSION = 1


def write_checkpoint(root: str, sampler, propose_cov, chains=None, exchange=None, collector: dict | None = None,
                     history: bool = True, chain_collector=None) -> str:
    """Write ``root.chk`` atomically.  ``propose_cov``: the proposal covariance
    in force (n_used x n_used); ``collector``: any extra JSON-able run state
    (sample counters, MaxLike, burn-in flags ...); ``chain_collector``: a
    converge.ChainCollector whose host state is saved beside the device
    Samples lists of the image."""
    image = sampler.save_state()
    meta = {"W": sampler.W, "np": sampler.np, "params_used": list(sampler.params_used),
            "propose_cov": np.asarray(propose_cov, dtype=np.float64).tolist(),
            "collector": collector or {},
            "flukecheck": bool(exchange.flukecheck) if exchange is not None else False,
            "chains": chains.checkpoint_state(sampler.W) if chains is not None else None,
            "chain_collector": chain_collector.checkpoint_state() if chain_collector is not None else None}
    hist = b""
    if history and getattr(sampler, "_hist_cap", 0):
        count = sampler.history_count()
        first = max(0, count - sampler._hist_cap)
        meta["history"] = {"first": first, "count": count - first, "capacity": sampler._hist_cap}
        if count > first:
            hist = np.ascontiguousarray(sampler.history_host(first, count - first)).tobytes()
            if getattr(sampler, "_likes", None):
                meta["history"]["terms"] = len(sampler._likes)
                hist += np.ascontiguousarray(sampler.history_terms(first, count - first)).tobytes()
    js = json.dumps(meta).encode()
    tmp = root + ".chk_tmp"
    with open(tmp, "wb") as f:
        f.write(struct.pack("<ii", CHK_ID, VERSION))
        for part in (js, image, hist):
            f.write(struct.pack("<Q", len(part)))
            f.write(part)
    os.replace(tmp, root + ".chk")
    return root + ".chk"


def read_checkpoint(root: str, sampler, chains=None, exchange=None, theory_fn=None, chain_collector=None) -> dict:
    """Resume ``sampler`` (same configuration and likelihoods as the run that
    wrote the file) from ``root.chk``; returns the ``collector`` dict.
    chain_collector: a converge.ChainCollector built on ``sampler`` for the
    resumed run before this call (the image carries its device Samples lists
    and load_state checks the capacity); its host state is restored.
    theory_fn: when the run moved slow parameters (step_theory / step_drag),
    the theory at the restored points is recomputed with it
    (BatchedMCMC.refresh_theory); without it stepping fails loudly."""
    with open(root + ".chk", "rb") as f:
        data = f.read()
    if len(data) < 8:
        raise ValueError(f"{root}.chk: invalid checkpoint file")
    cid, ver = struct.unpack_from("<ii", data, 0)
    if cid != CHK_ID:
        raise ValueError(f"{root}.chk: invalid checkpoint file")             # DoAbort, SampleCollector.f90:198
    if ver > VERSION:
        raise ValueError(f"{root}.chk: unknown checkpoint format {ver}")      # :158
    parts, off = [], 8
    for _ in range(3):
        (n,) = struct.unpack_from("<Q", data, off)
        parts.append(data[off + 8:off + 8 + n])
        off += 8 + n
    meta = json.loads(parts[0])
    if meta["W"] != sampler.W or meta["np"] != sampler.np or meta["params_used"] != list(sampler.params_used):
        raise ValueError(f"{root}.chk was written by a different sampler configuration")
    sampler.set_covariance(np.asarray(meta["propose_cov"]))
    sampler.load_state(parts[1])
    h = meta.get("history")
    if h is not None and getattr(sampler, "_hist_cap", 0):
        flat = np.frombuffer(parts[2], dtype=np.float64)
        if h["count"]:
            nr = h["count"] * (len(sampler.params_used) + 1) * sampler.W
            rows = flat[:nr].reshape(h["count"], len(sampler.params_used) + 1, sampler.W)
            terms = None
            if h.get("terms"):
                terms = flat[nr:].reshape(h["count"], h["terms"], sampler.W)
            keep = min(h["count"], sampler._hist_cap)
            sampler.history_restore(h["first"] + h["count"] - keep, rows[h["count"] - keep:],
                                    None if terms is None else terms[h["count"] - keep:])
        else:                                   # checkpoint taken before the first recorded step
            sampler.history_restore(h["first"], np.empty((0, len(sampler.params_used) + 1, sampler.W)))
    if chains is not None and meta.get("chains") is not None:
        chains.restore(meta["chains"], sampler.W)
    if exchange is not None:
        exchange.flukecheck = meta["flukecheck"]
    if chain_collector is not None:
        if meta.get("chain_collector") is None:
            raise ValueError(f"{root}.chk holds no ChainCollector state")
        chain_collector.restore(meta["chain_collector"])
    if theory_fn is not None:
        sampler.refresh_theory(theory_fn)
    return meta["collector"]
