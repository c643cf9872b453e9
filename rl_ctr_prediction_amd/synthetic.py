"""Synthetic Criteo-shape CTR batches.

F fields in one global id space of V ids. Per-field cardinality is skewed like Criteo's
categorical columns: the first 4 fields hold 80% of V, the next 6 hold 19%, the rest 1%.
Within a field ids follow a truncated Zipf(1.1) law mapped through a fixed permutation
(so hot ids are scattered over the table, not clustered at the field start). Labels come
from a planted FM (std 0.01, 4 latent dims, hash-generated so no table is materialised)
shifted to a CTR of about 0.25. Everything is seeded: the same (seed, rank) gives the
same batches on every host.
"""
from __future__ import annotations

import math

import numpy as np

_SHARES = ((4, 0.80), (6, 0.19))  # (fields, share of V); the remaining fields share 1%


def field_cardinalities(V: int, F: int = 26) -> np.ndarray:
    shares = []
    left = F
    for nf, s in _SHARES:
        k = min(nf, left)
        shares += [s / nf] * k
        left -= k
    if left > 0:
        rest = 1.0 - sum(s for _, s in _SHARES[: len(shares)])
        shares += [max(rest, 0.01) / left] * left
    shares = np.asarray(shares[:F], dtype=np.float64)
    shares /= shares.sum()
    card = np.maximum(1, np.floor(shares * V).astype(np.int64))
    card[0] += V - card.sum()  # exact total
    if card[0] < 1:
        raise ValueError(f"V={V} too small for F={F} fields")
    return card


def _mix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    return x


def _gauss_hash(ids: np.ndarray, salt: int) -> np.ndarray:
    h = _mix64(ids.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(salt))
    u1 = ((h >> np.uint64(11)).astype(np.float64) + 0.5) / float(1 << 53)
    h2 = _mix64(h + np.uint64(0x632BE59BD9B4E019))
    u2 = ((h2 >> np.uint64(11)).astype(np.float64) + 0.5) / float(1 << 53)
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * math.pi * u2)


class CriteoSynth:
    def __init__(self, V: int, F: int = 26, zipf_s: float = 1.1, seed: int = 1,
                 uniform: bool = False):
        self.V, self.F, self.s, self.uniform = int(V), int(F), float(zipf_s), uniform
        self.card = field_cardinalities(self.V, self.F)
        self.offset = np.concatenate([[0], np.cumsum(self.card)[:-1]])
        self.seed = seed
        # per-field permutation multiplier coprime to the cardinality
        rng = np.random.default_rng(seed + 7777)
        self.mult = np.empty(self.F, dtype=np.int64)
        self.add = np.empty(self.F, dtype=np.int64)
        for f in range(self.F):
            n = int(self.card[f])
            m = int(rng.integers(1, max(2, n))) | 1
            while math.gcd(m, n) != 1:
                m += 2
            self.mult[f] = m % max(n, 1) if n > 1 else 0
            self.add[f] = int(rng.integers(0, n))

    def ids(self, rng: np.random.Generator, n: int) -> np.ndarray:
        out = np.empty((n, self.F), dtype=np.int64)
        a = 1.0 - self.s
        for f in range(self.F):
            c = int(self.card[f])
            u = rng.random(n)
            if self.uniform:
                rank = np.minimum((u * c).astype(np.int64), c - 1)
            else:  # inverse CDF of the continuous power law on [1, c+1)
                r = (((c + 1.0) ** a - 1.0) * u + 1.0) ** (1.0 / a)
                rank = np.clip(np.floor(r).astype(np.int64) - 1, 0, c - 1)
            local = (rank * int(self.mult[f]) + int(self.add[f])) % c
            out[:, f] = self.offset[f] + local
        return out

    def planted_logit(self, x: np.ndarray) -> np.ndarray:
        """The planted FM's logit of each example, without the CTR shift (float64 [B])."""
        w = 0.01 * _gauss_hash(x, 1)
        z = w.sum(axis=1)
        s = np.zeros(x.shape[0])
        q = np.zeros(x.shape[0])
        for d in range(4):
            v = 0.01 * _gauss_hash(x, 100 + d)
            s_d = v.sum(axis=1)
            s += s_d * s_d
            q += (v * v).sum(axis=1)
        return z + 0.5 * (s - q)

    def labels(self, rng: np.random.Generator, x: np.ndarray) -> np.ndarray:
        w = 0.01 * _gauss_hash(x, 1)
        z = np.full(x.shape[0], math.log(0.25 / 0.75))
        z += w.sum(axis=1)
        s = np.zeros(x.shape[0])
        q = np.zeros(x.shape[0])
        for d in range(4):
            v = 0.01 * _gauss_hash(x, 100 + d)
            s_d = v.sum(axis=1)
            s += s_d * s_d
            q += (v * v).sum(axis=1)
        z += 0.5 * (s - q)
        p = 1.0 / (1.0 + np.exp(-z))
        return (rng.random(x.shape[0]) < p).astype(np.float32)

    def batches(self, n_batches: int, B: int, rank: int = 0):
        rng = np.random.default_rng([self.seed, rank])
        for _ in range(n_batches):
            x = self.ids(rng, B)
            yield x, self.labels(rng, x)

    def batch(self, i: int, B: int, rank: int = 0):
        """Batch i of an independently seeded stream (seed, rank, i): any batch can be
        generated on its own, so a long stream is produced in parallel."""
        rng = np.random.default_rng([self.seed, rank, 1 << 20, i])
        x = self.ids(rng, B)
        return x, self.labels(rng, x)

    def stream(self, n_batches: int, B: int, rank: int = 0, threads: int = 8, start: int = 0):
        """Batches start .. start + n_batches - 1 of batch(), generated on `threads` threads
        (numpy releases the GIL in the bulk array work)."""
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max(1, threads)) as ex:
            return list(ex.map(lambda i: self.batch(i, B, rank), range(start, start + n_batches)))
