#!/usr/bin/env python3
"""Generate docs/metrics.md from the PRODUCT: every row is a family the native exporter rendered
in one of the configurations below, so the reference can never list a family the exporter does not
emit, or miss one it does (tests/test_fuzz_and_fleet.py::test_metrics_doc_matches_the_product
checks both directions, against the family literals in csrc/ too).

Configurations (all native, no Python oracle):
* core       -- mock backend with every table field filled (`full=1`), processes, allocations,
                RAS events, two ticks (interval-rate families need a second table);
* control    -- the same exporter's native metadata pollers against a fake kubelet (CRI +
                PodResources), a fake Docker daemon and a kubelet log tree + device-plugin checkpoint;
* influx     -- the batched Influx push against a local sink;
* pmc/probe/helper -- the on-device samplers through the fake plugins, in the helper process
                (csrc/fakes/fake_ondevice.cpp; `make fakes`);
* http_rt_priority -- SCHED_FIFO HTTP loops (their self-metrics);
* amdsmi     -- the libamd_smi backend over the fake library (backend-specific self-metrics).
"""

import json
import os
import sys
import tempfile
import threading
import time
from http.server import BaseHTTPRequestHandler, HTTPServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))  # fake kubelet / Docker servers (test fixtures)

REFERENCE = {
    "node_gpu_gpu_util": "node_gpu.gpu_util (gpu.py:138)",
    "node_gpu_mem_util": "node_gpu.mem_util (gpu.py:133-135,139)",
    "node_gpu_mem_used": "node_gpu.mem_used (gpu.py:139)",
    "node_gpu_mem_total": "node_gpu.mem_total (gpu.py:139-140)",
    "node_gpu_mem_free": "node_gpu.mem_free (gpu.py:143)",
    "node_gpu_mem_bw_util": "utilization.memory, queried but dropped (gpu.py:105)",
    "pod_gpu_used_memory": "pod_gpu.used_memory (gpu.py:204,216; idle rows gpu.py:239,250)",
    "pod_gpu_gpu_util": "pod_gpu.gpu_util (device-wide, gpu.py:205,215)",
    "pod_gpu_allocated": "pod_gpu.count by user_name_t (2019 dashboard)",
    "gpumon_gpus": "GPU总数 / 已占GPU数量 / 占GPU未开始使用 / 占GPU已使用完毕 stat panels",
}

CONTROL_PREFIXES = ("gpumon_cri_", "gpumon_podresources_", "gpumon_docker_", "gpumon_kubelet_files_")


class _Sink(BaseHTTPRequestHandler):
    def do_POST(self):  # noqa: N802
        self.rfile.read(int(self.headers.get("Content-Length", 0)))
        self.send_response(204)
        self.end_headers()

    def log_message(self, *a):
        pass


def _kubelet_tree(d):
    logs = os.path.join(d, "log")
    os.makedirs(os.path.join(logs, "pods", "ml_jupyter-q-0_uid-1", "c"))
    os.makedirs(os.path.join(logs, "containers"))
    os.symlink("/var/log/pods/ml_jupyter-q-0_uid-1/c/0.log",
               os.path.join(logs, "containers", f"jupyter-q-0_ml_c-{'a' * 64}.log"))
    ckpt = os.path.join(d, "ckpt")
    with open(ckpt, "w") as fh:
        json.dump({"Data": {"PodDeviceEntries": [
            {"PodUID": "uid-1", "ContainerName": "c", "ResourceName": "amd.com/gpu", "DeviceIDs": {"0": ["x"]},
             "AllocResp": ""}]}, "Checksum": 1}, fh)
    return logs, ckpt


def _families(ex):
    from gpumon.export import promtext

    return promtext.parse(ex.metrics_text())


def collect():
    """{family: (type, help, labels, source)} over every configuration."""
    from gpumon import core
    from gpumon.config import Config
    from oracles.attribution.fake_kubelet import FakeKubelet
    from test_docker import FakeDocker

    c = core()
    out = {}

    def add(fam, source):
        for name, f in fam.items():
            if name in out:
                continue
            labels = set()
            for _, l, _ in f["samples"]:
                labels |= {k for k in l if k != "le"}
            src = source(name) if callable(source) else source
            out[name] = (f["type"], f["help"], sorted(labels), src)

    srv = HTTPServer(("127.0.0.1", 0), _Sink)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    with tempfile.TemporaryDirectory() as d:
        logs, ckpt = _kubelet_tree(d)
        with FakeKubelet(podres_socket=f"{d}/kubelet.sock", cri_socket=f"{d}/cri.sock") as k, \
                FakeDocker(f"{d}/docker.sock", []) as dk:
            ex = c.Exporter({"backend": "mock:gpus=1,full=1", "serve_http": False, "interval_s": 0, "host": "node",
                             "cri_socket": k.cri_socket, "pod_resources_socket": k.podres_socket,
                             "docker_socket": dk.path, "pod_log_root": logs, "device_checkpoint": ckpt,
                             "influx_url": f"http://127.0.0.1:{srv.server_port}/write?db=k8s", "ras_every": 1})
            ex.start()
            try:
                ex.mock_set_procs([{"pid": os.getpid(), "device": 0, "name": "python", "vram_bytes": 1 << 30,
                                    "queues": 2}])
                ex.set_allocations([{"pod_namespace": "ml", "pod_name": "jupyter-q-0", "container_name": "c",
                                     "gpu_index": 0}])
                ex.mock_set_ras_event(0, "bad_pages", 0.0)
                ex.tick()
                time.sleep(0.05)  # past one firmware refresh (20 ms): interval rates need a new table
                ex.tick()
                deadline = time.time() + 5  # the Influx pusher posts from its own thread
                while "gpumon_influx_push_total" not in _families(ex) and time.time() < deadline:
                    time.sleep(0.02)
                base = _families(ex)
                add(base, lambda n: "control plane" if n.startswith(CONTROL_PREFIXES)
                    else "influx push" if n.startswith("gpumon_influx") else "core")
                # the on-device samplers exactly as deployed: the helper process runs the (fake) plugins
                plug = os.path.join(ROOT, "build", "fakes", "ondevice")
                # the default counter set plus SQ_WAVE_CYCLES (gpu_occupancy_percent, opt-in)
                od = c.OnDevice(ex, {"plugin_dir": plug, "pmc": True, "probe": True, "pmc_every_s": 60,
                                     "probe_every_s": 60, "pmc_window_s": 0.01, "ondevice_isolate": True,
                                     "pmc_counters": Config().pmc_counters + ["SQ_WAVE_CYCLES"]})
                od.start()
                od.step()
                ex.tick()
                add(_families(ex), lambda n: "probe" if n.startswith("gpu_probe") else
                    "helper" if n.startswith("gpumon_ondevice") else "pmc")
                od.stop()
            finally:
                ex.stop()
    srv.shutdown()
    # HTTP loops at SCHED_FIFO (http_rt_priority): their self-metrics
    ex = c.Exporter({"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                     "host": "node", "http_rt_priority": 1})
    if ex.start() == "":
        ex.tick()
        add(_families(ex), "http_rt_priority")
    ex.stop()
    # gzip scrapes on every tick: the snapshot compression counters (eager after 4 of 8 gzip-scraped ticks)
    import urllib.request

    ex = c.Exporter({"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0, "host": "node"})
    ex.start()
    for _ in range(8):
        ex.tick()
        req = urllib.request.Request(f"http://127.0.0.1:{ex.port}/metrics", headers={"Accept-Encoding": "gzip"})
        urllib.request.urlopen(req, timeout=5).read()
    ex.tick()
    add(_families(ex), "gzip scrapes")
    ex.stop()
    # /metrics over HTTPS (tls_cert_file): the handshake-failure counter; a throwaway certificate
    import shutil
    import subprocess

    if shutil.which("openssl"):
        with tempfile.TemporaryDirectory() as d:
            subprocess.run(["openssl", "req", "-x509", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1",
                            "-nodes", "-days", "1", "-keyout", f"{d}/k.pem", "-out", f"{d}/c.pem", "-subj", "/CN=node"],
                           check=True, capture_output=True, timeout=60)
            ex = c.Exporter({"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                             "host": "node", "tls_cert_file": f"{d}/c.pem", "tls_key_file": f"{d}/k.pem"})
            ex.start()
            ex.tick()
            add(_families(ex), "tls_cert_file")
            ex.stop()
            # mutual TLS (tls_client_ca_file): the client-certificate refusal counter
            ex = c.Exporter({"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                             "host": "node", "tls_cert_file": f"{d}/c.pem", "tls_key_file": f"{d}/k.pem",
                             "tls_client_ca_file": f"{d}/c.pem"})
            ex.start()
            ex.tick()
            add(_families(ex), "tls_client_ca_file")
            ex.stop()
    # /metrics behind a bearer token (http_auth_token_file)
    with tempfile.TemporaryDirectory() as d:
        with open(f"{d}/token", "w") as f:
            f.write("doc-token\n")
        ex = c.Exporter({"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                         "host": "node", "http_auth_token_file": f"{d}/token"})
        ex.start()
        ex.tick()
        add(_families(ex), "http_auth_token_file")
        ex.stop()
    # backend-specific self-metrics: the libamd_smi backend over the fake library
    saved = os.environ.get("FAKE_AMDSMI_GPUS")  # the fake reads it at init; leave the caller's env as it was
    os.environ["FAKE_AMDSMI_GPUS"] = "1"
    try:
        ex = c.Exporter({"backend": "amdsmi", "amdsmi_lib": os.path.join(ROOT, "build", "fakes", "libfake_amd_smi.so"),
                         "serve_http": False, "interval_s": 0, "host": "node", "verify_kfd": False})
        if ex.start() == "":
            ex.tick()
            add(_families(ex), "amdsmi backend")
        ex.stop()
    finally:
        if saved is None:
            os.environ.pop("FAKE_AMDSMI_GPUS", None)
        else:
            os.environ["FAKE_AMDSMI_GPUS"] = saved
    return out


def build() -> str:
    rows = collect()
    out = ["# Metric reference", "",
           "Generated by `tools/gen_metrics_doc.py` from the native exporter's own expositions (mock backend",
           "with every field filled, the metadata pollers against fake kubelet / Docker endpoints, the Influx",
           "push, the on-device samplers through the fake plugins, the libamd_smi backend over the fake",
           "library); do not edit by hand. `source` says which configuration emits a family.",
           "Device series carry `host` and `gpu_id` (the reference's tags, /root/reference/gpu.py:137);",
           "`gpu_info` carries `gpu_uuid`, `bdf`, model and partition (use `--full-device-labels` to put",
           "uuid/bdf on every series). A device family appears only while some GPU reports the field: on",
           "MI355X the fan and voltage fields are N/A and those families stay absent.", "",
           "Every family can be left out of `/metrics` with `metrics_exclude` (or served alone with",
           "`metrics_include`): shell globs on the family name, e.g. `metrics_exclude: [gpu_xcd_*]`. On an",
           "8-GPU node that drops the per-XCD series, 448 of 1469 sample lines and 34 KB of a 118 KB body",
           "(mock backend). The Influx push keeps the reference's fixed layout. A scrape can filter for",
           "itself with the same globs: `/metrics?include=node_gpu_*,gpu_up` or `?exclude=gpu_xcd_*`",
           "(comma-separated, repeatable, percent-decoded), e.g. a fast Prometheus job for the reference",
           "families next to a slow one for everything (`params:` in the scrape config).", "",
           "| metric | type | source | labels | reference equivalent | help |", "|---|---|---|---|---|---|"]
    for name, (typ, help_, labels, src) in rows.items():
        out.append(f"| `{name}` | {typ} | {src} | {', '.join(labels)} | {REFERENCE.get(name, '[new]')} | "
                   f"{help_.replace('|', '/')} |")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    text = build()
    path = os.path.join(ROOT, "docs", "metrics.md")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    if len(sys.argv) > 1 and sys.argv[1] == "--check":
        sys.exit(0 if open(path).read() == text else 1)
    open(path, "w").write(text)
    print(path)
