"""HIP ordinal <-> exporter device, matched by PCI BDF.

A process that loads GPUs names them by HIP ordinal, and under ``HIP_VISIBLE_DEVICES=3,5`` (or
``ROCR_VISIBLE_DEVICES``, or a container runtime that exposes a subset of the node) ordinals
0 and 1 are the node's GPUs 3 and 5. The exporter's ``gpu_id`` is libamd_smi's node-wide
``hip_id`` (rocm_smi fallback: its enumeration index), so ``range(n)`` on both sides silently
pairs the wrong GPUs whenever the visible set is not a prefix of the node. Both sides agree on the
PCI address: ``hipDeviceGetPCIBusId`` here, ``amdsmi_get_gpu_device_bdf`` / ``rsmi_dev_pci_id_get``
in the exporter, whose ``devices`` filter accepts BDFs (csrc/core/backend.h set_device_filter).

The reference numbered GPUs by nvidia-smi output order (``shortunitids``,
/root/reference/gpu.py:119-120) and never had to pair them with a loader.
"""

from __future__ import annotations

import re
from typing import Dict, Iterable, List, Sequence

_BDF = re.compile(r"^(?:([0-9a-fA-F]{1,4}):)?([0-9a-fA-F]{1,2}):([0-9a-fA-F]{1,2})\.([0-7])$")


class DeviceMapError(RuntimeError):
    """A loaded GPU that the exporter does not sample (or samples twice)."""


def normalize_bdf(s: str) -> str:
    """"dddd:bb:dd.f" in lower case, domain 0000 when missing; "" when ``s`` is not a BDF. Same
    rule as the native normalize_bdf (csrc/core/common.cpp)."""
    m = _BDF.match((s or "").strip())
    if not m:
        return ""
    dom, bus, dev, fn = (int(x, 16) if x else 0 for x in m.groups())
    if dev > 0x1F:
        return ""
    return f"{dom:04x}:{bus:02x}:{dev:02x}.{fn:x}"


def hip_bdfs(ordinals: Iterable[int]) -> Dict[int, str]:
    """BDF of each HIP ordinal as this process sees it (gpumon._hip.device_pci_bus_id)."""
    from .._native import hip

    H = hip()
    out = {}
    for o in ordinals:
        b = normalize_bdf(H.device_pci_bus_id(int(o)))
        if not b:
            raise DeviceMapError(f"HIP ordinal {o}: no PCI bus id")
        out[int(o)] = b
    return out


def kfd_bdfs(ordinals: Iterable[int], topology: str = "/sys/class/kfd/kfd/topology/nodes",
             env: Dict[str, str] | None = None) -> Dict[int, str]:
    """The BDF each HIP ordinal WILL have, read from KFD's topology without initialising HIP (so
    a child process can be started first): the runtime enumerates the GPU nodes (gpu_id != 0) in
    node order, then ``ROCR_VISIBLE_DEVICES`` and ``HIP_VISIBLE_DEVICES`` (numeric lists) each
    select and reorder. Ordinals it cannot predict (a UUID-valued variable, fewer nodes) are left
    out; :func:`hip_bdfs` after initialisation is the check."""
    import os

    env = os.environ if env is None else env
    nodes = []
    try:
        names = sorted((n for n in os.listdir(topology) if n.isdigit()), key=int)
    except OSError:
        return {}
    for n in names:
        try:
            with open(f"{topology}/{n}/gpu_id") as fh:
                if int(fh.read().strip() or 0) == 0:
                    continue  # a CPU node
            props = {}
            with open(f"{topology}/{n}/properties") as fh:
                for line in fh:
                    k, _, v = line.partition(" ")
                    props[k] = v.strip()
            loc, dom = int(props["location_id"]), int(props.get("domain", "0"))
        except (OSError, ValueError, KeyError):
            continue  # outside this container's device cgroup, or not a GPU with a PCI location
        nodes.append(f"{dom:04x}:{(loc >> 8) & 0xFF:02x}:{(loc >> 3) & 0x1F:02x}.{loc & 0x7:x}")
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
        sel = env.get(var)
        if sel is None or sel.strip() == "":
            continue
        try:
            nodes = [nodes[int(x)] for x in sel.split(",") if x.strip()]
        except (ValueError, IndexError):
            return {}  # UUIDs or an index past the end: no prediction
    return {int(o): nodes[int(o)] for o in ordinals if 0 <= int(o) < len(nodes)}


def match(ordinal_bdfs: Dict[int, str], statics: Sequence[dict], replicas: bool = False) -> List[dict]:
    """One row per loaded ordinal: ``{hip_ordinal, bdf, gpu_id, index}`` where ``index`` is the
    exporter's device index (the position in ``samples()`` / ``rates()``) of the GPU with that
    BDF. Raises :class:`DeviceMapError` if a BDF matches no sampled device or several -- unless
    ``replicas`` (the ``amdsmi:replicate=R`` rehearsal samples each GPU R times): then the first."""
    by_bdf: Dict[str, List[dict]] = {}
    for s in statics:
        b = normalize_bdf(s.get("bdf", ""))
        if b:
            by_bdf.setdefault(b, []).append(s)
    rows = []
    for o in sorted(ordinal_bdfs):
        b = normalize_bdf(ordinal_bdfs[o])
        hits = by_bdf.get(b, [])
        if replicas and hits:
            hits = hits[:1]
        if len(hits) != 1:
            have = sorted(by_bdf)
            raise DeviceMapError(f"HIP ordinal {o} (BDF {b or ordinal_bdfs[o]!r}) matches {len(hits)} "
                                 f"exporter device(s); the exporter samples {have}")
        s = hits[0]
        rows.append({"hip_ordinal": o, "bdf": b, "gpu_id": s.get("gpu_id", str(s.get("hip_id", ""))),
                     "index": int(s["index"])})
    return rows


def positional(n: int, statics: Sequence[dict]) -> List[dict]:
    """Rows for a backend with no PCI identity behind it (the mock): ordinal k = device k."""
    if len(statics) < n:
        raise DeviceMapError(f"exporter samples {len(statics)} device(s), {n} needed")
    return [{"hip_ordinal": k, "bdf": statics[k].get("bdf", ""), "gpu_id": statics[k].get("gpu_id", str(k)),
             "index": int(statics[k]["index"])} for k in range(n)]


def index_of(rows: Sequence[dict]) -> Dict[int, int]:
    """HIP ordinal -> exporter device index."""
    return {r["hip_ordinal"]: r["index"] for r in rows}


def exporter_rows(ex, ordinals: Iterable[int]) -> List[dict]:
    """:func:`match` of this process's HIP ordinals against a started exporter ``ex``."""
    return match(hip_bdfs(ordinals), ex.statics())
