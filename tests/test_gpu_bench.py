"""bench.py's device helpers on the GPU: the zero-copy archive view RCCL sends from."""
import importlib.util
import os

import numpy as np
import pytest
import torch

import cusz_amd as cz
from cusz_amd import datagen
from gpu_util import d2h

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_archive_view_is_the_archive():
    b = _bench()
    dims = (256, 40, 24)
    x = datagen.smooth3d_torch(dims, seed=4)
    r = cz.Resource(cz.F4, dims, stream=torch.cuda.current_stream().cuda_stream)
    ptr, nb, _ = r.compress(x.data_ptr(), 1e-4)
    view, scratch = b.archive_view(ptr, nb, x.device, None)
    assert view.numel() == nb and view.dtype == torch.uint8
    np.testing.assert_array_equal(view.cpu().numpy(), d2h(ptr, nb))
    print("zero-copy" if view.data_ptr() == ptr else "copied")
    r.close()
