"""Host-side helpers of the HIP boundary that run without a GPU."""
from __future__ import annotations

import collections

import pytest

from rl_ctr_prediction_amd import hip_ops


@pytest.mark.parametrize("n_cus", [256, 128, 512])
@pytest.mark.parametrize("frac", [0.125, 0.5, 0.625, 0.75, 1.0])
def test_cu_mask_words_balanced_over_xcds(n_cus, frac):
    """ctr_stream_create_cu_masked's mask (hip_ops.cu_mask_words): round(8 * frac) / 8 of the
    CUs, the same share on every XCD under either CU numbering the driver may use (XCD by
    XCD, or round robin over the 8 XCDs: tools/cumask_probe.hip found the latter), for CU
    counts that are multiples of 64 (MI355X: 256)."""
    words = hip_ops.cu_mask_words(n_cus, frac)
    assert len(words) == (n_cus + 31) // 32
    kept = [c for c in range(n_cus) if words[c // 32] >> (c % 32) & 1]
    q = round(8 * frac)
    assert len(kept) == n_cus * q // 8
    per = n_cus // 8
    for xcd_of in (lambda c: c // per, lambda c: c % 8):
        counts = collections.Counter(xcd_of(c) for c in kept)
        assert sorted(counts) == list(range(8))
        assert max(counts.values()) - min(counts.values()) == 0
    assert all(w < (1 << 32) for w in words)
