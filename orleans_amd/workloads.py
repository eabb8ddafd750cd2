"""Synthetic workloads for the benches and tests (no datasets: there is no network).

Data generation only -- no routing logic lives here.
"""
from __future__ import annotations

import numpy as np


def power_law_graph(n_nodes: int, mean_deg: float, seed: int, max_deg: int = 1 << 16, alpha: float = 2.5):
    """Synthetic follower graph for cfg 4: power-law follower counts (Pareto tail,
    exponent ``alpha``, capped at ``max_deg``), followers distinct within a row and never
    the publisher itself -- the shape ``AddFollower`` keeps (one dictionary key per
    follower).  Row u's followers are (u + 1 + S[(r_u + k) % L]) mod n for k < deg(u),
    with S a fixed sample of L distinct offsets in [0, n-1): distinct by construction.
    Returns (row_off u32[n+1], dst u32[E])."""
    rng = np.random.default_rng(seed)
    raw = (rng.pareto(alpha - 1.0, size=n_nodes) + 1.0)
    # P(deg >= x) ~ x^(1 - alpha); scale so that E[deg] = mean_deg before the cap (rounded)
    deg = np.minimum(np.floor(raw * (mean_deg * (alpha - 2.0) / (alpha - 1.0)) + 0.5).astype(np.int64), max_deg)
    deg = np.minimum(deg, n_nodes - 1)
    row_off = np.zeros(n_nodes + 1, dtype=np.int64)
    np.cumsum(deg, out=row_off[1:])
    if row_off[-1] >= 1 << 32:
        raise ValueError("graph too large for u32 edge offsets")
    L = int(min(n_nodes - 1, max(max_deg, 1)))
    S = rng.choice(n_nodes - 1, size=L, replace=False).astype(np.int64)
    r = rng.integers(0, L, size=n_nodes)
    E = int(row_off[-1])
    item = np.repeat(np.arange(n_nodes, dtype=np.int64), deg)
    k = np.arange(E, dtype=np.int64) - row_off[item]
    dst = ((item + 1 + S[(r[item] + k) % L]) % n_nodes).astype(np.uint32)
    return row_off.astype(np.uint32), dst


def zipf_cdf(n_grains: int, s: float = 1.1) -> np.ndarray:
    """Normalised Zipf(s) CDF over ranks 0..n_grains-1 (rank r has weight (r+1)^-s)."""
    cdf = np.cumsum(np.arange(1, n_grains + 1, dtype=np.float64) ** -s)
    return cdf / cdf[-1]


def zipf_ranks_np(n_grains: int, n: int, seed: int, s: float = 1.1) -> np.ndarray:
    """n grain ranks ~ Zipf(s) by inverse CDF (SURVEY 8 d cfg 3), on the host."""
    rng = np.random.default_rng(seed)
    return np.minimum(np.searchsorted(zipf_cdf(n_grains, s), rng.random(n)), n_grains - 1).astype(np.int64)


def zipf_keys_torch(tcd: int, n_grains: int, n: int, seed: int, dev, s: float = 1.1):
    """(n, 3) int64 GrainId keys on `dev`: grain k ~ Zipf(s) over ranks 0..n_grains-1 by inverse
    CDF, sampled on the GPU (BASELINE cfg 3); grain k is GrainId(type, k): [0, k, tcd]."""
    import torch
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    cdf = torch.arange(1, n_grains + 1, dtype=torch.float64, device=dev).pow_(-s).cumsum_(0)
    cdf /= cdf[-1].clone()
    u = torch.rand(n, dtype=torch.float64, device=dev, generator=gen)
    k = torch.searchsorted(cdf, u).clamp_(max=n_grains - 1)
    del cdf, u
    keys = torch.zeros((n, 3), dtype=torch.int64, device=dev)
    keys[:, 1] = k
    keys[:, 2] = int(np.uint64(tcd).astype(np.int64))
    return keys


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def mixed_grain_keys(tcds, n_grains: int, guid_every: int = 100) -> np.ndarray:
    """(n_grains, 3) u64 keys of a mixed directory: grain g is of class
    tcds[g % len(tcds)]; every guid_every-th grain is Guid-keyed (UniqueKey.NewKey(Guid), category
    Grain: N0 and N1 from the Guid's bytes, UniqueKey.cs:135-143 -- here a splitmix64 stream, N0 != 0),
    the others long-keyed (GrainId.GetGrainId(typeCode, g): N0 = 0, N1 = g, GrainId.cs:72-77)."""
    g = np.arange(n_grains, dtype=np.uint64)
    out = np.zeros((n_grains, 3), dtype=np.uint64)
    out[:, 1] = g
    out[:, 2] = np.asarray(tcds, dtype=np.uint64)[(g % np.uint64(len(tcds))).astype(np.int64)]
    if guid_every:
        sel = (g % np.uint64(guid_every)) == np.uint64(guid_every - 1)
        out[sel, 0] = _splitmix64(g[sel] * np.uint64(2) + np.uint64(1)) | np.uint64(1)
        out[sel, 1] = _splitmix64(g[sel] * np.uint64(2) + np.uint64(2))
    return out


def grain_keys_torch(tcd: int, ks, dev):
    """(n, 3) int64 keys [0, k, tcd] on `dev` for a 1-D tensor (or range) of long keys."""
    import torch
    ks = torch.as_tensor(ks, device=dev, dtype=torch.int64)
    keys = torch.zeros((ks.shape[0], 3), dtype=torch.int64, device=dev)
    keys[:, 1] = ks
    keys[:, 2] = int(np.uint64(tcd).astype(np.int64))
    return keys
