"""The histogram fold (GRS_OPT_FOLD, include/grs.h): the upfront histogram kernel counts pass
0's digit only, and each pass counts the next pass's digit of the keys it ranks and adds the
tile's counts into that pass's histogram rows (grs_pass.hpp PassFold).  Every pass kernel and
tile shape must give the exact stable sort with it, including ragged last tiles (their
all-ones padding keys are not counted), bit ranges whose last digit is narrower than 8 bits,
and a sorter that switches the fold on and off between calls."""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

SHAPES = [
    (32, False, {}),                                    # small tiles below one big tile per CU
    (32, False, {"tile": "big"}),                       # big tiles (v4, or v6 on small grids)
    (32, False, {"tile": "big", "pass": "v6"}),         # persistent
    (32, False, {"tile": "big", "xl": "always"}),       # XL two-round tiles
    (32, True, {"tile": "big"}),                        # u32 pairs: record passes
    (32, True, {"tile": "big", "xl": "always"}),
    (64, False, {"tile": "big"}),                       # u64: 8 passes, 7 folds
    (64, True, {"tile": "big"}),                        # u64 pairs: two-round big tiles
    (32, False, {"tile": "big", "rank": "match"}),      # ballot-match fallback
]


def _keys(n, key_bits, seed):
    k = oracle.splitmix_keys(n, key_bits, seed)
    k[::17] = np.iinfo(k.dtype).max            # genuine all-ones keys beside the padding
    return k


def _check(gpu, s, keys, pairs, end_bit=None):
    sk = keys if end_bit is None else keys & ((1 << end_bit) - 1)
    perm = np.argsort(sk, kind="stable")
    k = torch.from_numpy(keys).to(gpu)
    v = torch.arange(keys.size, dtype=torch.int64, device=gpu).to(torch.uint32) if pairs else None
    s.sort(k, v, end_bit=end_bit)
    s.check_error()
    assert np.array_equal(k.cpu().numpy(), keys[perm])
    if pairs:
        assert np.array_equal(v.cpu().numpy(), perm.astype(np.uint32))


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: f"{s[0]}{'p' if s[1] else ''}-"
                         + "-".join(f"{a}={b}" for a, b in s[2].items()))
@pytest.mark.parametrize("n", [1, 4097, (1 << 20) + 3, 9_437_185])
def test_fold_exact(gpu, shape, n):
    import gpuradixsort_amd as grs

    key_bits, pairs, opts = shape
    s = grs.RadixSorter(n, key_bits=key_bits, pairs=pairs, options=dict(opts, fold="on"))
    _check(gpu, s, _keys(n, key_bits, n + key_bits), pairs)


@pytest.mark.parametrize("end_bit", [20, 27, 32])
def test_fold_bit_ranges(gpu, end_bit):
    """Bits [0, end_bit): the last pass's digit is 4 or 3 bits wide (the fold's next-digit
    mask), or a full byte."""
    import gpuradixsort_amd as grs

    n = 3_000_017
    s = grs.RadixSorter(n, key_bits=32, pairs=True, options={"fold": "on", "tile": "big"})
    _check(gpu, s, _keys(n, 32, end_bit), True, end_bit)


def test_fold_toggles_between_calls(gpu):
    """The control blocks alternate between calls (each call's histogram kernel zeroes the next
    one's rows): switching the fold on and off between sorts must stay exact."""
    import gpuradixsort_amd as grs

    n = 5_000_011
    s = grs.RadixSorter(n, key_bits=32)
    for i, mode in enumerate(["on", "off", "on", "on", "off", "on"]):
        s.set_option("fold", mode)
        _check(gpu, s, _keys(n, 32, 100 + i), False)
