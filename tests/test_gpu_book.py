"""The device codebook (book_device.hh, psz_amd_build_book_device) against its serial
restatement in the oracle (orc_book_twoqueue_u2): book and reverse book byte for byte, on
random, skewed, sparse, tied, single-symbol and deep (Fibonacci: length-limited) histograms and
on a config-2 code histogram; its total bit count equals the reference heap's (both Huffman)."""
import numpy as np
import pytest
import torch

import cusz_amd as cz
from gpu_util import sync

pytestmark = pytest.mark.gpu


def device_book(hist, bklen, smooth):
    d_h = torch.from_numpy(np.ascontiguousarray(hist, np.uint32).view(np.int32)).cuda()
    d_b = torch.zeros(bklen, dtype=torch.int32, device="cuda")
    d_r = torch.zeros(4 * 64 + 2 * bklen, dtype=torch.uint8, device="cuda")
    cz.build_book_device(d_h.data_ptr(), bklen, smooth, d_b.data_ptr(), d_r.data_ptr(),
                         torch.cuda.current_stream().cuda_stream)
    sync()
    return d_b.cpu().numpy().view(np.uint32), d_r.cpu().numpy()


def histograms():
    rng = np.random.default_rng(11)
    out = []
    for bklen in (1024, 512, 128, 2):
        out.append(("uniform", bklen, rng.integers(0, 1000, bklen)))
        g = np.exp(-np.abs(np.arange(bklen) - bklen / 2) / (bklen / 40))
        out.append(("laplace", bklen, np.floor(g * 1e6).astype(np.int64)))
        sp = np.zeros(bklen, np.int64)
        idx = rng.choice(bklen, size=max(1, bklen // 20), replace=False)
        sp[idx] = rng.integers(1, 50, idx.size)
        out.append(("sparse", bklen, sp))
        out.append(("ties", bklen, np.full(bklen, 7)))
    one = np.zeros(1024, np.int64)
    one[300] = 12345
    out.append(("single", 1024, one))
    out.append(("empty", 1024, np.zeros(1024, np.int64)))
    fib = np.zeros(1024, np.int64)
    a, b = 1, 1
    for i in range(40):  # a Fibonacci histogram: Huffman depth 39 > 27 (halving path)
        fib[i * 7] = a
        a, b = b, a + b
    out.append(("fibonacci", 1024, fib))
    out.append(("huge", 1024, rng.integers(0, 2 ** 32 - 1, 1024, dtype=np.int64)))
    return out


@pytest.mark.parametrize("smooth", [0, 1])
def test_device_book_equals_oracle(oracle, smooth):
    for name, bklen, h in histograms():
        h = np.asarray(h, np.uint32)
        b_d, r_d = device_book(h, bklen, smooth)
        b_o, r_o = oracle.book_twoqueue(h, bklen, smooth)
        np.testing.assert_array_equal(b_d, b_o, err_msg=f"{name} bklen={bklen} smooth={smooth}: book")
        np.testing.assert_array_equal(r_d, r_o, err_msg=f"{name} bklen={bklen} smooth={smooth}: revbook")
        lens = b_d >> 27
        w = h.astype(np.int64) + smooth
        used = w > 0
        assert np.all((b_d[~used]) == 0xFFFFFFFF)
        if used.sum() >= 2:
            kraft = np.sum(2.0 ** -lens[used].astype(np.float64))
            assert kraft <= 1.0 + 1e-12 and lens[used].max() <= 27, name


def test_device_book_cost_equals_reference_heap(oracle):
    """Both are Huffman codes: the same total bits on the same histogram when no length limit
    applies (the heap's tie-breaking differs, the cost does not)."""
    rng = np.random.default_rng(5)
    for trial in range(20):
        h = np.floor(np.exp(-np.abs(np.arange(1024) - 512) / rng.uniform(2, 60)) * rng.uniform(1e3, 1e7))
        h = h.astype(np.uint32)
        b_d, _ = device_book(h, 1024, 0)
        b_r, _ = oracle.codebook(h, 1024)
        used = h > 0
        cost_d = int(np.sum(h[used].astype(np.int64) * (b_d[used] >> 27)))
        cost_r = int(np.sum(h[used].astype(np.int64) * (b_r[used] >> 27)))
        if (b_r[used] >> 27).max() < 27:
            assert cost_d == cost_r, trial
