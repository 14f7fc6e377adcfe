"""The raw-HSA probe path (csrc/plugins/probe_hsa.cpp) writes kernel arguments by hand: the layout
it writes must be the one the embedded gfx950 code object declares (csrc/hip/probe_co.hip), and the
bytes embedded in lib/libgpumon_probe.so must be that code object. CPU only: reads the ELF notes."""

import os
import subprocess

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HSACO = os.path.join(ROOT, "build", "obj", "hip", "probe_gfx950.hsaco")
LIB = os.path.join(ROOT, "lib", "libgpumon_probe.so")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"

# what probe_hsa.cpp writes: (offset, size) per argument, and the segment size it checks
EXPECTED = {
    "gpumon_probe_kernel": ([(0, 8), (8, 8), (16, 8), (24, 4), (28, 4), (32, 4)], 36),
    "gpumon_probe_reset": ([(0, 8), (8, 4)], 12),
}


def _kernels():
    if not (os.path.exists(HSACO) and os.path.exists(READELF)):
        pytest.skip("probe code object or llvm-readelf not built / installed")
    notes = subprocess.run([READELF, "--notes", HSACO], capture_output=True, text=True, check=True).stdout
    doc = yaml.safe_load(notes[notes.index("---"):notes.rindex("...")])  # the AMDGPU metadata is YAML
    return {k[".name"]: {"args": [(a[".offset"], a[".size"]) for a in k[".args"]],
                         "kernarg": k[".kernarg_segment_size"], "group": k[".group_segment_fixed_size"],
                         "private": k[".private_segment_fixed_size"], "wave": k[".wavefront_size"]}
            for k in doc["amdhsa.kernels"]}


def test_kernarg_layout_matches_the_hsa_dispatch():
    k = _kernels()
    for name, (args, seg) in EXPECTED.items():
        assert name in k, sorted(k)
        assert k[name]["args"] == args, (name, k[name]["args"])
        # no hidden (implicit) arguments: the hand-written block is the whole segment
        assert k[name]["kernarg"] == seg, (name, k[name]["kernarg"])
        assert k[name]["group"] == 0 and k[name]["private"] == 0 and k[name]["wave"] == 64


def test_library_embeds_this_code_object():
    if not (os.path.exists(HSACO) and os.path.exists(LIB)):
        pytest.skip("probe library not built")
    co = open(HSACO, "rb").read()
    assert co[:4] == b"\x7fELF"  # unbundled: hsa_code_object_reader_create_from_memory takes an ELF
    assert open(LIB, "rb").read().find(co) >= 0
