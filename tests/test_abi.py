"""CPU-only checks of the C-ABI library: it loads, exports every symbol that include/*.h
declares, and its structs have the reference's byte layout."""
import ctypes as C
import os
import re
import subprocess

import pytest

import cusz_amd as cz

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    names = set()
    for dp, _, fs in os.walk(os.path.join(ROOT, "include")):
        for f in fs:
            txt = open(os.path.join(dp, f)).read()
            txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
            txt = re.sub(r"static inline[^{]*\{.*?\n\}", "", txt, flags=re.S)
            for m in re.finditer(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", txt):
                name = m.group(1)
                if name not in ("sizeof", "if", "return"):
                    names.add(name)
    return names


def test_library_builds_and_loads():
    assert os.path.exists(cz.LIB_PATH), "run __graft_entry__.build() first"
    cz.lib()


def test_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", cz.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    declared = _declared_functions()
    assert declared, "header parse found nothing"
    missing = sorted(declared - exported)
    assert not missing, missing
    assert set(cz.EXPORTS) <= exported


def test_header_layout_matches_reference():
    h = cz.psz_header
    assert C.sizeof(h) == 176
    off = {f: getattr(h, f).offset for f, _ in h._fields_}
    assert off == {"dtype": 0, "pipeline": 4, "rc": 24, "vle_sublen": 48, "vle_pardeg": 52, "entry": 56,
                   "len": 80, "splen": 104, "user_input_eb": 112, "min_val": 120, "max_val": 128,
                   "intp_param": 136}
    assert C.sizeof(cz.psz_rc2) == 24 and C.sizeof(cz.psz_interp_params) == 40


def test_c_header_compiles_and_matches():
    """Compile a C program against include/ and check sizeof/offsetof like the reference."""
    src = r'''
#include <stddef.h>
#include <stdio.h>
#include "cusz.h"
#include "cusz_rev1.h"
#include "hf.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(psz_header), offsetof(psz_header, entry),
         offsetof(psz_header, splen), offsetof(psz_header, intp_param), sizeof(phf_header),
         offsetof(phf_header, entry));
  return 0;
}'''
    tmp = "/tmp/cusz_amd_abi_check"
    with open(tmp + ".c", "w") as f:
        f.write(src)
    subprocess.run(["gcc", "-std=c11", "-I" + os.path.join(ROOT, "include"), "-o", tmp, tmp + ".c"], check=True)
    out = subprocess.run([tmp], capture_output=True, text=True, check=True).stdout.split()
    assert out == ["176", "56", "104", "136", "64", "40"]
