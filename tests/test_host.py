"""Host-side checks that need no GPU: the C-ABI library loads, exports every symbol
include/cpr_hip.h declares, and its struct layouts match the ctypes mirrors."""

import ctypes
import pathlib
import re
import subprocess

import pytest

from cpr_amd import _lib as L

ROOT = pathlib.Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "cpr_hip.h"


def _declared():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\S.*?\b(cpr_[a-z_0-9]+)\(", text, flags=re.M)))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(str(L.LIB_PATH))
    declared = _declared()
    assert len(declared) >= 19
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(L.EXPORTS) == declared


def test_version_and_registry():
    lib = L.lib()
    assert lib.cpr_abi_version() == L.ABI_VERSION == 11
    assert lib.cpr_version().decode().startswith("cpr-hip")
    from cpr_amd import device

    # Collection.add prepends (collection.ml:13): reverse of nakamoto_ssz.ml:342-350
    assert [n for n, _ in device.policy_registry()] == [
        "sapirshtein-2016-sm1", "eyal-sirer-2014", "simple", "honest"]
    # bk_ssz.ml:404-415, same reversal
    assert [n for n, _ in device.policy_registry(L.PROTO_BK)] == [
        "avoid-loss", "minor-delay", "get-ahead", "honest"]


def test_struct_layouts_match_header(tmp_path):
    src = tmp_path / "sz.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "cpr_hip.h"\n'
        'int main(){printf("%zu %zu %zu %zu %zu\\n", sizeof(cpr_config), sizeof(cpr_episode_record),'
        ' sizeof(cpr_summary), sizeof(cpr_step_info), offsetof(cpr_config, seed));'
        'printf("%zu\\n", offsetof(cpr_config, k));return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), "-o", str(exe), str(src)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    want = [ctypes.sizeof(L.Config), ctypes.sizeof(L.EpisodeRecord), ctypes.sizeof(L.Summary),
            ctypes.sizeof(L.StepInfo), L.Config.seed.offset, L.Config.k.offset]
    assert got == want


def test_no_device_raises_loudly(monkeypatch):
    # without a HIP device the product path must fail, never fall back to the CPU
    import torch

    if torch.cuda.device_count() > 0:
        pytest.skip("a HIP device is present")
    from cpr_amd import device

    with pytest.raises(Exception):
        device.Context(0)


def _header_struct_fields(name):
    text = HEADER.read_text()
    body = re.search(r"typedef struct " + name + r" \{(.*?)\} " + name + ";", text, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        for part in re.sub(r"\[.*?\]", "", decl).split(","):
            fields.append(re.findall(r"[A-Za-z_][A-Za-z_0-9]*", part)[-1])
    return fields


def test_ocaml_bindings_follow_the_header():
    # integration/ocaml/cpr_hip.ml (not compiled here: no OCaml toolchain) must name every
    # struct field in header order and bind every exported function
    ml = (ROOT / "integration" / "ocaml" / "cpr_hip.ml").read_text()
    for struct, var in [("cpr_config", "config"), ("cpr_episode_record", "record"),
                        ("cpr_summary", "summary"), ("cpr_step_info", "step_info"),
                        ("cpr_trace", "trace")]:
        got = re.findall(r"field " + var + r' "([a-z_0-9]+)"', ml)
        assert got == _header_struct_fields(struct), struct
    bound = set(re.findall(r'foreign\s+"(cpr_[a-z_0-9]+)"', ml))
    assert bound == set(_declared())
    assert f"let abi_version = {L.ABI_VERSION}" in ml
