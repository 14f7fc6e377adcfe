"""Property tests of the renderers (hypothesis-generated label values and GPU/process sets) and a
fleet test: several node-local exporters scraped by one scraper (the reference's only
"distributed" mode: N independent DaemonSet pods, gpu_monitor.yaml:1-5; Prometheus does fan-in)."""

import os

from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from gpumon.export import promtext

label_text = st.text(alphabet=st.characters(blacklist_categories=("Cs",), blacklist_characters="\x00"),
                     min_size=1, max_size=40)


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(pod=label_text, ns=label_text, user=label_text, procname=label_text)
def test_pod_labels_roundtrip_any_text(core, pod, ns, user, procname):
    ex = core.Exporter({"backend": "mock:gpus=1", "serve_http": False, "interval_s": 0, "host": 'no"de\\1'})
    ex.start()
    try:
        ex.mock_set_procs([{"pid": 1, "device": 0, "name": procname, "vram_bytes": 7 << 20}])
        ex.set_allocations([{"pod_namespace": ns, "pod_name": pod, "container_name": "c", "gpu_index": 0,
                             "user_name": user}])
        ex.tick()
        fam = promtext.parse(ex.metrics_text())  # must stay valid exposition for any input
        idle = [l for _, l, _ in fam["pod_gpu_used_memory"]["samples"] if l["pid"] == "-"]
        assert idle and idle[0]["podname"] == pod and idle[0]["namespace"] == ns and idle[0]["user_name"] == user
        assert idle[0]["host"] == 'no"de\\1'
        procs = [l for _, l, _ in fam["pod_gpu_used_memory"]["samples"] if l["pid"] == "1"]
        assert procs and procs[0]["procressname"] == procname
        # Influx lines: one line per row, no raw newlines leaking into a line
        lines = ex.influx_text().split("\n")
        assert sum(l.startswith("pod_gpu,") for l in lines) == 2
    finally:
        ex.stop()


@settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(gpus=st.integers(0, 16), procs=st.lists(st.tuples(st.integers(1, 10**6), st.integers(0, 15)), max_size=30),
       unsupported=st.lists(st.sampled_from(["temp_hotspot", "power_cur", "vram_used", "xcd", "xgmi", "gfx_util"]),
                            max_size=4))
def test_any_device_and_process_set_renders_valid(core, gpus, procs, unsupported):
    spec = f"mock:gpus={gpus}" + (f",unsupported={';'.join(unsupported)}" if unsupported else "")
    ex = core.Exporter({"backend": spec, "serve_http": False, "interval_s": 0})
    ex.start()
    try:
        ex.mock_set_procs([{"pid": p, "device": d} for p, d in procs])
        ex.tick()
        fam = promtext.parse(ex.metrics_text())
        n = len(promtext.values(fam, "gpu_up"))
        assert n == gpus
        seen = {(p, d) for p, d in procs if d < gpus}
        assert len(promtext.values(fam, "pod_gpu_used_memory_bytes")) == len(seen)
    finally:
        ex.stop()


def test_fleet_of_exporters_one_scraper(core):
    nodes = []
    try:
        for i in range(3):
            ex = core.Exporter({"backend": f"mock:gpus={2 + i}", "listen_addr": "127.0.0.1", "port": 0,
                                "interval_s": 0.05, "host": f"gpu-node-{i}", "http_threads": 1})
            ex.start()
            nodes.append(ex)
        total = {}
        for ex in nodes:
            r = core.scrape_load("127.0.0.1", ex.port, "/metrics", n_requests=20, concurrency=2)
            assert r["errors"] == 0
            fam = promtext.parse(ex.metrics_text())
            for _, labels, v in fam["gpumon_gpus"]["samples"]:
                if labels["state"] == "total":
                    total[labels["host"]] = v
        assert total == {"gpu-node-0": 2, "gpu-node-1": 3, "gpu-node-2": 4}
    finally:
        for ex in nodes:
            ex.stop()


def test_metrics_doc_is_current():
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    from conftest import make_locked

    make_locked("fakes")  # the on-device rows come from the fake plugins
    r = subprocess.run([sys.executable, os.path.join(root, "tools/gen_metrics_doc.py"), "--check"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, "docs/metrics.md is stale: run python tools/gen_metrics_doc.py"


# String literals in csrc/ that look like family names but are not: label keys, libamd_smi call
# names (gpumon_backend_call_* labels), a sysfs file name, and the on-device plugins' dlsym'd ABI
# symbols (csrc/plugins/ondevice_abi.h).
NOT_FAMILIES = {"gpu_id", "gpu_uuid", "gpu_metrics", "gpu_activity", "gpu_vram_bad_pages",
                # JSON keys of the loopback /debug views (csrc/core/exporter_debug.cpp)
                "gpu_util", "process_list_failures"}
NOT_FAMILY_PREFIXES = ("gpumon_pmc_abi", "gpumon_pmc_agent", "gpumon_pmc_init", "gpumon_pmc_read_running",
                       "gpumon_pmc_sample_many", "gpumon_pmc_stop_running", "gpumon_probe_abi", "gpumon_probe_create",
                       "gpumon_probe_destroy", "gpumon_probe_device_count", "gpumon_probe_device_pci", "gpumon_probe_launch",
                       "gpumon_probe_wait")


def test_metrics_doc_matches_the_product():
    """docs/metrics.md lists exactly what the native exporter emits. Each row's
    family is a literal in the C++ sources (nothing harvested from test oracles), and each
    family-shaped literal in csrc/core and csrc/plugins is a row, unless it is a declared
    non-family string."""
    import glob
    import re

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    doc = open(os.path.join(root, "docs", "metrics.md")).read()
    rows = set(re.findall(r"^\| `([a-z0-9_]+)` \|", doc, re.M))
    src = ""
    for f in glob.glob(os.path.join(root, "csrc", "core", "*.cpp")) + glob.glob(os.path.join(root, "csrc", "plugins", "*.cpp")):
        src += open(f).read()
    literals = set(re.findall(r'"((?:gpu|gpumon|node_gpu|pod_gpu|process)_[a-z0-9_]+)"', src))
    assert rows and rows <= literals, sorted(rows - literals)
    families = {x for x in literals if x not in NOT_FAMILIES and not x.startswith(NOT_FAMILY_PREFIXES)}
    assert families <= rows, sorted(families - rows)
    assert not any(x in rows for x in ("gpumon_control_plane_up", "gpumon_control_plane_refresh_seconds"))


def test_configuration_doc_is_current():
    import importlib.util

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("gen_config_doc", os.path.join(root, "tools/gen_config_doc.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    with open(os.path.join(root, "docs/configuration.md")) as fh:
        assert fh.read() == mod.render(), "docs/configuration.md is stale: run python tools/gen_config_doc.py"
