"""Wire-format compatibility: archives a reference encoder writes -- the
CPU oracle assembles them in the reference layout (chunks in index order, no gaps) at the
chunk lengths the reference's coarse tuning picks on different GPUs -- decompress through the
C API (psz_decompress_float) and through the CLI (`cusz -x`), bit for bit equal to the oracle's
reconstruction.  The decoder reads chunk c at par_entry[c] with the header's sublen
(hf_kernels.cuhip.inl:384-392, hf_buf.cc:199-211); the CLI loads the stored file
(cli.cc:122-163)."""
import subprocess

import numpy as np
import pytest

import cusz_amd as cz
from archive_util import oracle_archive
from cusz_amd import datagen
from gpu_util import d2h, sync, to_device

pytestmark = pytest.mark.gpu

EB = 1e-4
FIELDS = {
    "1d": (lambda: datagen.hacc1d_np(100_003, 7), (100_003, 1, 1)),
    "2d": (lambda: datagen.cesm2d_np((300, 200), 7), (300, 200, 1)),
    "3d": (lambda: datagen.smooth3d_np((64, 48, 40), 7), (64, 48, 40)),
    "3d_brickwidth": (lambda: datagen.smooth3d_np((512, 24, 16), 7), (512, 24, 16)),
}


def _archive(oracle, name, sublen):
    make, dims = FIELDS[name]
    data = make()
    codes, ov, oi = oracle.lorenzo_c(data, dims, EB)
    book, rv = oracle.codebook(oracle.histogram(codes))
    arch = oracle_archive(oracle, codes, ov, oi, dims, EB, book, rv, sublen=sublen)
    want = oracle.lorenzo_x(codes, ov, oi, dims, EB)
    return data, dims, arch, want


@pytest.mark.parametrize("sublen", [256, 2048, 4864])
@pytest.mark.parametrize("name", list(FIELDS))
def test_decompress_oracle_archive(oracle, name, sublen):
    data, dims, arch, want = _archive(oracle, name, sublen)
    h = cz.psz_header.from_buffer_copy(arch[:176])
    r = cz.Resource(cz.F4, None, header=h)
    d_arch = to_device(np.frombuffer(arch, np.uint8))
    out = to_device(np.full(want.size, np.nan, np.float32))  # not pre-zeroed
    r.decompress(d_arch.data_ptr(), len(arch), out.data_ptr())
    sync()
    got = d2h(out.data_ptr(), 4 * want.size, np.float32)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    ulp = 2.0 ** -23 * float(np.abs(data).max())  # f32 rounding of the reconstruction
    assert np.abs(got.astype(np.float64) - data).max() <= 1.001 * EB + ulp


@pytest.mark.parametrize("name,sublen", [("1d", 2048), ("2d", 4864), ("3d", 256), ("3d_brickwidth", 256)])
def test_cli_decompresses_oracle_archive(oracle, tmp_path, name, sublen):
    data, dims, arch, want = _archive(oracle, name, sublen)
    f = tmp_path / "field.f32"
    data.tofile(f)
    (tmp_path / "field.f32.cusza").write_bytes(arch)
    x = subprocess.run([cz.CLI_PATH, "-x", "-i", str(tmp_path / "field.f32.cusza"), "--origin", str(f)],
                       capture_output=True, text=True, timeout=120)
    assert x.returncode == 0, x.stderr
    got = np.fromfile(tmp_path / "field.f32.cuszx", dtype=np.float32)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
