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


@pytest.mark.parametrize("cname,pyname", [("dmx_config", "Config"), ("dmx_stats", "Stats")])
def test_struct_layout_matches_header(tmp_path, cname, pyname):
    """The ctypes mirrors in dmx.py have the C header's field offsets and size (a field added
    to one side only would shift every later field)."""
    import ctypes
    py = getattr(dmx, pyname)
    fields = [f[0] for f in py._fields_]
    src = tmp_path / "layout.c"
    body = "".join(f'printf("{f} %zu\\n", offsetof({cname}, {f}));' for f in fields)
    src.write_text("#include <stddef.h>\n#include <stdio.h>\n#include <dmx.h>\n"
                   f'int main(void){{{body} printf("sizeof %zu\\n", sizeof({cname})); return 0;}}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", f"-I{ROOT}/include", str(src), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], check=True, capture_output=True,
                                                        text=True).stdout.splitlines())
    for f in fields:
        assert int(got[f]) == getattr(py, f).offset, f
    assert int(got["sizeof"]) == ctypes.sizeof(py)
    hdr = open(os.path.join(ROOT, "include", "dmx.h")).read()
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (cname, cname), hdr, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    cfields = re.findall(r"\b([a-z_][a-z0-9_]*)\s*;", body)
    assert cfields == fields


def test_config_defaults_and_dev_controls():
    """dmx_config_default: one device, 32 KiB segments, no flags, the developer controls off; the
    Python mirror maps its developer keywords onto those fields (no device needed)."""
    import ctypes
    cfg = dmx.Config()
    dmx.lib().dmx_config_default(ctypes.byref(cfg))
    assert (cfg.device, cfg.segment_bytes, cfg.flags, cfg.n_gpus) == (-1, 32768, 0, 1)
    assert (cfg.dev_inflate_pass, cfg.dev_heavy_bytes) == (0, 0)
    assert dmx.DMX_CFG_FB_SERIAL == 2 and dmx.DMX_CFG_RFC_STRICT == 1
    hdr = open(os.path.join(ROOT, "include", "dmx.h")).read()
    assert re.search(r"#define DMX_CFG_FB_SERIAL 2u", hdr)
