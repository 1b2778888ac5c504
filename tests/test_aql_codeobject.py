"""The code object the engine dispatches its joins from (gochugaru_amd/csrc/aql.inc): built beside
libgck.so, it holds the kernels aql.inc looks up by their demangled names, and their kernarg
segments have the layout aql_dispatch writes — the by-value parameters from offset 0, then the code
object v5 hidden block counts at the next 8-byte boundary, the group sizes 12 bytes later and the
grid dimensions at +64. No GPU needed: the metadata notes are read with llvm-readelf."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CO = os.path.join(ROOT, "gochugaru_amd", "libgck_kernels.co")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"

# demangled name (as aql.inc looks it up) -> sizes of the by-value parameters
KERNELS = {
    "void gck::k_label_join<24, 16u, 32u, false>(gck::LjArgs)": [248],
    "void gck::k_label_join<24, 32u, 32u, false>(gck::LjArgs)": [248],
    "void gck::k_label_join<32, 16u, 32u, false>(gck::LjArgs)": [248],
    "void gck::k_label_join<32, 32u, 32u, false>(gck::LjArgs)": [248],
    "void gck::k_label_join<24, 16u, 32u, true>(gck::LjArgs)": [248],
    "void gck::k_label_join<24, 32u, 32u, true>(gck::LjArgs)": [248],
    "void gck::k_label_join<32, 16u, 32u, true>(gck::LjArgs)": [248],
    "void gck::k_label_join<32, 32u, 32u, true>(gck::LjArgs)": [248],
    "void gck::k_closure_join<24, 2048u, 32u, true>(gck::Ctx, gck::CjArgs)": [344, 184],
}


def _kernels():
    if not os.path.exists(CO):
        pytest.skip("libgck_kernels.co not built")
    if not os.path.exists(READELF):
        pytest.skip("llvm-readelf missing")
    notes = subprocess.run([READELF, "--notes", CO], capture_output=True, text=True, check=True).stdout
    out, cur = {}, None
    # the metadata is YAML-like: per kernel an .args list, then .name
    for block in notes.split("  - .agpr_count:")[1:]:
        name = re.search(r"\.name:\s+(\S+)", block).group(1)
        args = [(int(o), int(s), k) for o, s, k in
                re.findall(r"\.offset:\s+(\d+)\s+\.size:\s+(\d+)\s+\.value_kind:\s+(\w+)", block)]
        ks = int(re.search(r"\.kernarg_segment_size:\s+(\d+)", block).group(1))
        out[name] = (args, ks)
    return out


def _demangle(names):
    cf = shutil.which("c++filt")
    if not cf:
        pytest.skip("c++filt missing")
    res = subprocess.run([cf], input="\n".join(names), capture_output=True, text=True, check=True).stdout
    return dict(zip(res.splitlines(), names))


def test_dispatched_kernels_present_with_their_kernarg_layout():
    ks = _kernels()
    by_dm = _demangle(list(ks))
    for dm, sizes in KERNELS.items():
        assert dm in by_dm, f"{dm} not in the code object"
        args, seg = ks[by_dm[dm]]
        explicit = [a for a in args if a[2] == "by_value"]
        assert [s for _, s, _ in explicit] == sizes, (dm, explicit)
        off = 0
        for (o, s, _), want in zip(explicit, sizes):
            assert o == off, (dm, o, off)
            off += s
        hid = (off + 7) & ~7
        kinds = {k: o for o, _, k in args}
        assert kinds.get("hidden_block_count_x") == hid, (dm, kinds)
        assert kinds.get("hidden_group_size_x") == hid + 12, (dm, kinds)
        if "hidden_grid_dims" in kinds:
            assert kinds["hidden_grid_dims"] == hid + 64, (dm, kinds)
        assert seg == hid + 256 and seg <= 1024, (dm, seg)  # the whole hidden block; aql.inc kAqlKernargBytes


def test_code_object_carries_the_build_id():
    """aql.inc kBuildId: the code object exports the variable aql_init compares with the library's."""
    if not os.path.exists(CO) or not os.path.exists(READELF):
        pytest.skip("code object or llvm-readelf missing")
    syms = subprocess.run([READELF, "--syms", CO], capture_output=True, text=True, check=True).stdout
    assert "gck_kernels_build_id" in syms
