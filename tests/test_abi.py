"""CPU: the C-ABI library loads and exports every symbol include/dmx.h declares; the drop-in
headers compile against it.  No GPU work is launched here."""
import os
import re
import subprocess

import pytest

import dmx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "dmx.h")).read()
    return sorted(set(re.findall(r"\b(dmx_[a-z0-9_]+)\s*\(", hdr)))


def test_every_declared_symbol_is_exported():
    lib = dmx.lib()
    syms = declared_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(dmx.EXPORTS) == syms


def test_bound_and_strerror():
    assert dmx.deflate_bound(0) >= 2
    for n in (1, 100, 32768, 1 << 30):
        assert dmx.deflate_bound(n) >= n + 10 * -(-n // 32768) + 5
    assert dmx.strerror(dmx.DMX_ERR_OVERREAD) == "Reading bits beyond the alloted buffer size!"


def test_no_cpu_fallback_without_device():
    """On a host without a gfx950 GPU, creating a context fails loudly (DMX_ERR_DEVICE)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(dmx.DmxError) as e:
        dmx.Context()
    assert e.value.code == dmx.DMX_ERR_DEVICE


def test_dropin_headers_compile(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text('#include <deflate.hpp>\n#include <inflate.hpp>\nint main(){return 0;}\n')
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror", f"-I{ROOT}/include", str(src)],
                   check=True)


def test_dropin_program_links():
    exe = os.path.join(ROOT, "tests", "cpp", "dropin_test")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)
    assert os.path.exists(exe)
