"""Static checks of the deployment artefacts (no cluster needed).

Reference manifest (/root/reference/gpu_monitor.yaml) used extensions/v1beta1 with no selector,
probes, resources or ports and mounted the host docker socket; these tests pin the replacements.
"""

import json
import os
import re
import time

import pytest
import yaml

from gpumon.export import promtext

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _docs(path):
    with open(os.path.join(ROOT, path)) as fh:
        return [d for d in yaml.safe_load_all(fh) if d]


def test_daemonset_is_apps_v1_and_complete():
    docs = _docs("deploy/k8s/gpumon-daemonset.yaml")
    kinds = {d["kind"]: d for d in docs}
    assert set(kinds) == {"ConfigMap", "DaemonSet", "Service"}
    ds = kinds["DaemonSet"]
    assert ds["apiVersion"] == "apps/v1"
    sel = ds["spec"]["selector"]["matchLabels"]
    tpl = ds["spec"]["template"]
    assert all(tpl["metadata"]["labels"][k] == v for k, v in sel.items())
    spec = tpl["spec"]
    assert spec["hostPID"] is True
    assert any(t["key"] == "CriticalAddonsOnly" for t in spec["tolerations"])  # reference toleration
    c = spec["containers"][0]
    env = {e["name"]: e for e in c["env"]}
    assert env["NODE_NAME"]["valueFrom"]["fieldRef"]["fieldPath"] == "spec.nodeName"  # reference env
    assert c["ports"][0]["containerPort"] == 9400
    assert c["readinessProbe"]["httpGet"]["path"] == "/readyz"
    assert c["livenessProbe"]["httpGet"]["path"] == "/healthz"
    mounts = {m["mountPath"] for m in c["volumeMounts"]}
    assert "/var/lib/kubelet/pod-resources" in mounts
    assert "/var/run/docker.sock" not in mounts and "/usr/bin/docker" not in mounts
    assert tpl["metadata"]["annotations"]["prometheus.io/port"] == "9400"


def test_configmap_keys_are_valid_config():
    from gpumon.config import Config

    cm = [d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "ConfigMap"][0]
    data = yaml.safe_load(cm["data"]["config.yaml"])["gpumon"]
    Config().apply_dict(data)  # raises on unknown keys


def test_servicemonitor():
    sm = _docs("deploy/k8s/gpumon-servicemonitor.yaml")[0]
    assert sm["kind"] == "ServiceMonitor"
    assert sm["spec"]["endpoints"][0]["port"] == "metrics"
    # /readyz is 503 while the device backend is down: the Service must still list the pod, or the
    # series that say why (gpumon_backend_up 0, the GpumonExporterDown alert) are never scraped
    svc = next(d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "Service")
    assert svc["spec"]["publishNotReadyAddresses"] is True


def _plugin_metric_names():
    names = set()
    for f in os.listdir(os.path.join(ROOT, "gpumon/ops")):
        if f.endswith(".py"):
            names |= set(re.findall(r'"(gpu_[a-z0-9_]+)"', open(os.path.join(ROOT, "gpumon/ops", f)).read()))
    # the production on-device samplers (native)
    names |= set(re.findall(r'"((?:gpu|gpumon)_[a-z0-9_]+)"', open(os.path.join(ROOT, "csrc/core/ondevice.cpp")).read()))
    return names


def test_dashboard_queries_resolve_against_exposition(mock_exporter):
    """Every metric a dashboard panel queries is produced by the exporter (mock scrape) or by one
    of the optional device plugins (probe kernel / PMC)."""
    import subprocess
    import sys

    subprocess.run([sys.executable, os.path.join(ROOT, "deploy/grafana/make_dashboard.py")], check=True,
                   stdout=subprocess.DEVNULL)
    dash = json.load(open(os.path.join(ROOT, "deploy/grafana/gpumon-dashboard.json")))
    ex = mock_exporter(backend="mock:gpus=2")
    ex.set_allocations([{"pod_namespace": "ml", "pod_name": "jupyter-e-0", "container_name": "c", "gpu_index": 0}])
    ex.mock_set_procs([{"pid": os.getpid(), "device": 1, "name": "python3"}])
    ex.mock_set_occ_series(1, [100.0])
    ex.set_device_mfma_util({1: 50.0})  # what the PMC sampler publishes (pod_gpu_mfma_util_percent)
    time.sleep(0.05)  # past one firmware refresh (20 ms): interval rates need a new table
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    produced = set()
    for f, v in fam.items():
        produced.add(f)
        for n, _, _ in v["samples"]:
            produced.add(n)
    plugins = _plugin_metric_names() | _product_families()  # samplers, pollers, RT loops, amdsmi backend
    words = {"sum", "by", "count", "rate", "increase", "max", "histogram_quantile", "le", "host", "user_name", "link",
             "gpu_id", "state", "m", "s", "time", "result"}
    missing = []
    titles = []
    for p in dash["panels"]:
        titles.append(p["title"])
        for t in p["targets"]:
            for name in re.findall(r"\b([a-z_][a-z0-9_]*)\s*[{(\[]", t["expr"]):
                if name in words:
                    continue
                if name not in produced and name not in plugins:
                    missing.append((p["title"], name))
    assert not missing, missing
    # reference panels recreated
    for t in ["GPU总数", "已占GPU数量", "占GPU未开始使用", "占GPU已使用完毕", "当前使用显存", "GPU使用率",
              "容器使用GPU情况", "每个用户占用GPU的数量"]:
        assert any(t in x for x in titles), t


def test_dockerfile_entrypoint():
    """the image runs the native exporter (no Python in the runtime stage), from a
    plain base plus the staged closure (deploy/image_closure.py; tests/test_image_closure.py)."""
    txt = open(os.path.join(ROOT, "deploy/Dockerfile")).read()
    runtime = txt.split("\nFROM ${BASE_IMAGE}", 1)[1]
    assert 'ENTRYPOINT ["/opt/gpumon/bin/gpumon-exporter"]' in runtime
    assert 'CMD ["--config", "/etc/gpumon/config.yaml"]' in runtime
    assert "ARG BASE_IMAGE=ubuntu:22.04" in txt
    assert "python" not in runtime.lower() and "pip" not in runtime and "apt-get" not in runtime
    assert "COPY --from=build /rootfs/ /" in runtime
    assert "image_closure.py stage --root /rootfs --overlays" in txt
    assert "libltdl" not in txt.split("\n", 5)[-1] or "no vendored" in txt
    assert "EXPOSE 9400" in txt and "GPUMON_PLUGIN_DIR=/opt/gpumon/lib" in runtime


def _build_stage_copies(dockerfile):
    """(sources, dest) of every COPY in the Dockerfile's first (build) stage, in order. Only the
    plain `COPY src... dest` form (no --from, no heredocs) may appear there."""
    copies, stage = [], 0
    for line in open(dockerfile).read().splitlines():
        words = line.split()
        if not words:
            continue
        if words[0] == "FROM":
            stage += 1
            if stage > 1:
                break
        elif words[0] == "COPY" and stage == 1:
            assert not any(w.startswith("--") for w in words[1:]), line
            copies.append((words[1:-1], words[-1]))
    assert copies, "no COPY in the build stage"
    return copies


def _stage_tree(copies, dst):
    """What `docker build` would see: each COPY source from a clean checkout (tracked files only,
    so in-tree build outputs such as gpumon/_core*.so do not hide a missing rule)."""
    import shutil
    import subprocess

    tracked = None
    if os.path.isdir(os.path.join(ROOT, ".git")):
        out = subprocess.run(["git", "-C", ROOT, "ls-files"], capture_output=True, text=True, check=True).stdout
        tracked = set(out.split())
    for srcs, dest in copies:
        for s in srcs:
            target = os.path.normpath(os.path.join(dst, dest if not dest.endswith("/") and len(srcs) == 1
                                                   and dest not in ("./", ".") else os.path.join(dest, s)))
            src = os.path.join(ROOT, s)
            if os.path.isdir(src):
                for base, _, files in os.walk(src):
                    for f in files:
                        rel = os.path.relpath(os.path.join(base, f), ROOT)
                        if tracked is not None and rel not in tracked:
                            continue
                        if tracked is None and (f.endswith((".so", ".o", ".pyc")) or "__pycache__" in rel):
                            continue
                        out = os.path.join(target, os.path.relpath(os.path.join(base, f), src))
                        os.makedirs(os.path.dirname(out), exist_ok=True)
                        shutil.copy2(os.path.join(base, f), out)
            else:
                os.makedirs(os.path.dirname(target), exist_ok=True)
                shutil.copy2(src, target)


def _make_targets(dockerfile):
    m = re.search(r"^RUN make\b(.*)$", open(dockerfile).read(), re.M)
    assert m, "the build stage runs make"
    return [w for w in m.group(1).split() if not w.startswith("-")]


def test_image_build_stage_makes_all_from_its_copy_set(tmp_path):
    """deploy/Dockerfile's build stage must build from exactly the files it
    COPYs. `make -n all` over that set resolves every prerequisite (a rule that needs tools/ or
    tests/ fails here), and `make core` really compiles there. Reference: its image builds from the
    two files it ADDs (/root/reference/Dockerfile:1-7)."""
    import subprocess

    df = os.path.join(ROOT, "deploy", "Dockerfile")
    copies = _build_stage_copies(df)
    _stage_tree(copies, str(tmp_path))
    assert sorted(os.listdir(tmp_path)) == ["Makefile", "csrc", "deploy", "gpumon"], sorted(os.listdir(tmp_path))
    assert os.listdir(tmp_path / "deploy") == ["image_closure.py"]
    targets = _make_targets(df)
    assert targets == ["all", "GPUMON_ARCH=gfx950"], targets
    r = subprocess.run(["make", "-C", str(tmp_path), "-n", *targets], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "tools/" not in r.stdout and "tests/" not in r.stdout
    r = subprocess.run(["make", "-C", str(tmp_path), "-j8", "core"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert os.path.exists(tmp_path / "bin" / "gpumon-exporter")


def test_copy_set_check_catches_an_outside_prerequisite(tmp_path):
    """The check above is not vacuous: the same COPY set with `all` depending on a tools/ target
    (round 3's `snapshot`) fails `make -n all`."""
    import subprocess

    _stage_tree(_build_stage_copies(os.path.join(ROOT, "deploy", "Dockerfile")), str(tmp_path))
    mk = (tmp_path / "Makefile").read_text()
    mk = re.sub(r"^all:(.*)$", r"all:\1 bin/perf_snapshot_probe", mk, count=1, flags=re.M)
    (tmp_path / "Makefile").write_text(mk)
    r = subprocess.run(["make", "-C", str(tmp_path), "-n", "all", "GPUMON_ARCH=gfx950"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "tools/perf_snapshot_probe.hip" in r.stderr, (r.returncode, r.stderr[-500:])


def _product_families():
    """Every family the native exporter emits in the metric reference's configurations (mock with
    full tables, CRI / PodResources / Docker / kubelet-files pollers, Influx push, on-device samplers
    through the helper, the amdsmi backend): tools/gen_metrics_doc.py collect()."""
    import importlib.util

    from conftest import make_locked

    make_locked("fakes")
    spec = importlib.util.spec_from_file_location("gen_metrics_doc", os.path.join(ROOT, "tools", "gen_metrics_doc.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    fams = mod.collect()
    assert {"gpumon_cri_up", "gpumon_podresources_up", "gpumon_docker_up", "gpumon_kubelet_files_up"} <= set(fams)
    return set(fams)


def test_alert_and_recording_rules_resolve(mock_exporter):
    """Every series a PrometheusRule expression uses is produced by the exporter, and the label
    values the alerts match on (sensor, kind, state) exist in a scrape."""
    (rule,) = _docs("deploy/k8s/gpumon-alerts.yaml")
    assert rule["apiVersion"] == "monitoring.coreos.com/v1" and rule["kind"] == "PrometheusRule"
    ex = mock_exporter(backend="mock:gpus=2,mode=load")
    ex.set_allocations([{"pod_namespace": "ml", "pod_name": "p-0", "container_name": "c", "gpu_index": 0}])
    ex.mock_set_procs([{"pid": os.getpid(), "device": 1, "name": "python3"}])
    ex.tick()
    import time

    time.sleep(0.05)
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    produced = {n for f, v in fam.items() for n in [f] + [s[0] for s in v["samples"]]}
    produced |= _product_families()  # on-device samplers, metadata pollers, Influx push, amdsmi backend
    words = {"sum", "by", "count", "rate", "increase", "delta", "avg", "max", "time", "host", "namespace", "podname",
             "gpu_id", "user_name", "on"}
    exprs = [r["expr"] for g in rule["spec"]["groups"] for r in g["rules"]]
    assert len(exprs) >= 12
    for e in exprs:
        for name in re.findall(r"\b([a-z_][a-z0-9_]*)\s*[{(\[]", e) + re.findall(r"\b(gpu[a-z0-9_]*|pod_gpu[a-z0-9_]*|node_gpu[a-z0-9_]*)\b", e):
            if name in words:
                continue
            assert name in produced, (e, name)
    label_values = {(k, v) for f in fam.values() for _, labels, _ in f["samples"] for k, v in labels.items()}
    for k, v in [("sensor", "hotspot"), ("sensor", "mem"), ("kind", "socket_thermal"), ("kind", "hbm_thermal"),
                 ("kind", "vr_thermal"), ("state", "idle"), ("type", "uncorrectable"), ("type", "correctable"),
                 ("event", "poison_consumption"), ("event", "fatal")]:
        assert (k, v) in label_values, (k, v)
    kust = _docs("deploy/k8s/kustomization.yaml")[0]
    for r in kust["resources"]:
        assert os.path.exists(os.path.join(ROOT, "deploy/k8s", r)), r


def test_validation_job_and_tools_image():
    """The node-validation Job (reference Dockerfile2's debug-image role, made purpose-built) runs
    tools that exist in the tree, on the tools image, with the DaemonSet's device access."""
    (job,) = _docs("deploy/k8s/gpumon-validate-job.yaml")
    assert job["apiVersion"] == "batch/v1" and job["kind"] == "Job"
    spec = job["spec"]["template"]["spec"]
    assert spec["restartPolicy"] == "Never" and spec["hostPID"] is True
    (c,) = spec["containers"]
    assert c["image"].startswith("gpumon-tools:")
    script = c["args"][0]
    for tool in re.findall(r"(tools/[a-z_]+\.py|bench\.py)", script):
        assert os.path.exists(os.path.join(ROOT, tool)), tool
    mounts = {m["mountPath"] for m in c["volumeMounts"]}
    assert {"/sys", "/dev/kfd", "/dev/dri"} <= mounts
    txt = open(os.path.join(ROOT, "deploy/Dockerfile.tools")).read()
    assert "COPY tools /opt/gpumon/tools" in txt and "rocprofv3" in txt


@pytest.mark.parametrize("overlay,probe,blocks", [("ondevice", True, 3), ("pmc", False, 2)])
def test_ondevice_overlays_enable_their_samplers_and_size_limits(overlay, probe, blocks):
    """each on-device overlay turns on its samplers in a config the exporter accepts
    and sizes the pod for them: 0.11 GB + 173 MB per hardware queue per GPU on 8 GPUs -- PMC alone 2
    queues per GPU, PMC + probe 3 (profiles/r3_helper_memory.md, r3_probe_hsa.md) -- the same model
    the exporter exports as gpumon_ondevice_helper_memory_model_bytes."""
    from gpumon.config import Config

    (k,) = _docs(f"deploy/k8s/overlays/{overlay}/kustomization.yaml")
    assert k["resources"] == ["../../"]
    cfg_patch = next(p for p in k["patches"] if p["target"]["kind"] == "ConfigMap")
    value = yaml.safe_load(cfg_patch["patch"])[0]["value"]
    data = yaml.safe_load(value)["gpumon"]
    c = Config().apply_dict(data)
    assert c.enable_pmc and c.enable_probe is probe and c.ondevice_isolate and c.pmc_mode == "continuous"
    res_patch = next(p for p in k["patches"] if p["target"]["kind"] == "DaemonSet")
    res = yaml.safe_load(res_patch["patch"])[0]["value"]
    mib = int(res["limits"]["memory"].rstrip("Mi"))
    req = int(res["requests"]["memory"][:-2]) * (1024 if res["requests"]["memory"].endswith("Gi") else 1)
    model_mib = (110e6 + 8 * blocks * 173e6) / 2 ** 20
    assert model_mib <= req <= 1.1 * model_mib and 1.1 * req <= mib <= 1.35 * model_mib, (req, mib, model_mib)


def _json_patch(doc, ops):
    """The add / replace subset of RFC 6902 that the overlays use (kustomize applies the real one)."""
    import copy

    doc = copy.deepcopy(doc)
    for op in ops:
        keys = [k.replace("~1", "/").replace("~0", "~") for k in op["path"].lstrip("/").split("/")]
        parent = doc
        for k in keys[:-1]:
            parent = parent[int(k)] if isinstance(parent, list) else parent[k]
        last = keys[-1]
        if isinstance(parent, list):
            if op["op"] == "add":
                parent.insert(len(parent) if last == "-" else int(last), op["value"])
            else:
                parent[int(last)] = op["value"]
        else:
            assert op["op"] == "add" or last in parent, op["path"]
            parent[last] = op["value"]
    return doc


def test_ondevice_overlay_patches_apply_to_the_base_daemonset():
    """Every DaemonSet op of the overlay resolves against the base manifest, and every volume mount
    of the patched pod names a volume (the helper's runtimes get a writable /tmp under the base's
    read-only root filesystem)."""
    (k,) = _docs("deploy/k8s/overlays/ondevice/kustomization.yaml")
    ds = next(d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "DaemonSet")
    ops = yaml.safe_load(next(p for p in k["patches"] if p["target"]["kind"] == "DaemonSet")["patch"])
    out = _json_patch(ds, ops)
    pod = out["spec"]["template"]["spec"]
    vols = {v["name"] for v in pod["volumes"]}
    c = pod["containers"][0]
    assert all(m["name"] in vols for m in c["volumeMounts"])
    assert any(m["mountPath"] == "/tmp" for m in c["volumeMounts"]) and c["securityContext"]["readOnlyRootFilesystem"]
    assert c["resources"]["limits"]["memory"] == "5120Mi"


def test_docker_overlay_mounts_the_socket_and_sets_docker_socket():
    """Plain-Docker nodes (the reference's runtime, gpu_monitor.yaml:24-28): the opt-in overlay
    mounts the Docker socket where its config points the native Docker poller, and the base stays
    without it."""
    from gpumon.config import Config

    (k,) = _docs("deploy/k8s/overlays/docker/kustomization.yaml")
    assert k["resources"] == ["../../"]
    cfg_patch = next(p for p in k["patches"] if p["target"]["kind"] == "ConfigMap")
    c = Config().apply_dict(yaml.safe_load(yaml.safe_load(cfg_patch["patch"])[0]["value"])["gpumon"])
    assert c.docker_socket == "/var/run/docker.sock" and c.control_plane == "native"
    ds = next(d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "DaemonSet")
    ops = yaml.safe_load(next(p for p in k["patches"] if p["target"]["kind"] == "DaemonSet")["patch"])
    pod = _json_patch(ds, ops)["spec"]["template"]["spec"]
    vols = {v["name"]: v for v in pod["volumes"]}
    mounts = {m["mountPath"]: m for m in pod["containers"][0]["volumeMounts"]}
    assert all(m["name"] in vols for m in mounts.values())
    m = mounts[c.docker_socket]
    assert m["readOnly"] and vols[m["name"]]["hostPath"] == {"path": "/var/run/docker.sock", "type": "Socket"}
    base = ds["spec"]["template"]["spec"]["containers"][0]["volumeMounts"]
    assert all("docker" not in x["mountPath"] for x in base)


def test_influx_overlay_pushes_over_verified_https(core, tmp_path):
    """overlays/influx/: the reference's push on top of /metrics, for an InfluxDB 2.x / 3.x server
    over verified HTTPS. The token comes from a Secret, the server's CA from the same Secret
    (mounted), and the URL is one the exporter's startup check accepts."""
    import subprocess

    (k,) = _docs("deploy/k8s/overlays/influx/kustomization.yaml")
    assert k["resources"] == ["../../"]
    ds = next(d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "DaemonSet")
    ops = yaml.safe_load(next(p for p in k["patches"] if p["target"]["kind"] == "DaemonSet")["patch"])
    pod = _json_patch(ds, ops)["spec"]["template"]["spec"]
    c = pod["containers"][0]
    env = {e["name"]: e for e in c["env"]}
    assert env["INFLUXDB_TOKEN"]["valueFrom"]["secretKeyRef"] == {"name": "gpumon-influx", "key": "token"}
    assert "NODE_NAME" in env  # the base's env is kept
    url, ca = env["INFLUXDB_URL"]["value"], env["GPUMON_INFLUX_CA_FILE"]["value"]
    u = core.parse_url(url)
    assert u["ok"] and u["tls"] and "/api/v2/write?" in url, u
    vols = {v["name"]: v for v in pod["volumes"]}
    assert all(m["name"] in vols for m in c["volumeMounts"])
    m = next(m for m in c["volumeMounts"] if ca.startswith(m["mountPath"] + "/"))
    sec = vols[m["name"]]["secret"]
    assert m["readOnly"] and sec["secretName"] == "gpumon-influx"
    assert [i["path"] for i in sec["items"]] == [os.path.basename(ca)]
    # the startup check accepts that configuration once the Secret's CA file is there
    subprocess.run(["openssl", "req", "-x509", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes",
                    "-days", "1", "-keyout", str(tmp_path / "k"), "-out", str(tmp_path / "ca.crt"), "-subj", "/CN=ca"],
                   check=True, capture_output=True, timeout=60)
    assert core.check_push_config(url, token="tok", ca_file=str(tmp_path / "ca.crt")) == ""


def test_tls_overlay_serves_https_from_a_secret(core, tmp_path):
    """overlays/tls/: the exporter terminates TLS for /metrics. The certificate and key come from a
    Secret through GPUMON_TLS_* env. The probes switch to HTTPS, and the ServiceMonitor scrapes https
    and verifies against the Secret's CA. The files the env names are ones the startup check accepts."""
    import subprocess

    from gpumon.config import Config

    (k,) = _docs("deploy/k8s/overlays/tls/kustomization.yaml")
    ds = next(d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "DaemonSet")
    ops = yaml.safe_load(next(p for p in k["patches"] if p["target"]["kind"] == "DaemonSet")["patch"])
    pod = _json_patch(ds, ops)["spec"]["template"]["spec"]
    c = pod["containers"][0]
    env = {e["name"]: e.get("value") for e in c["env"]}
    cfg = Config().apply_env(env)
    assert cfg.tls_cert_file and cfg.tls_key_file
    assert c["readinessProbe"]["httpGet"]["scheme"] == "HTTPS" and c["livenessProbe"]["httpGet"]["scheme"] == "HTTPS"
    vols = {v["name"]: v for v in pod["volumes"]}
    assert all(m["name"] in vols for m in c["volumeMounts"])
    for f in (cfg.tls_cert_file, cfg.tls_key_file):
        m = next(m for m in c["volumeMounts"] if f.startswith(m["mountPath"] + "/"))
        assert m["readOnly"] and vols[m["name"]]["secret"]["secretName"] == "gpumon-tls"
    sm = next(d for d in _docs("deploy/k8s/gpumon-servicemonitor.yaml") if d["kind"] == "ServiceMonitor")
    sm_ops = yaml.safe_load(next(p for p in k["patches"] if p["target"]["kind"] == "ServiceMonitor")["patch"])
    ep = _json_patch(sm, sm_ops)["spec"]["endpoints"][0]
    assert ep["scheme"] == "https" and ep["tlsConfig"]["ca"]["secret"] == {"name": "gpumon-tls", "key": "ca.crt"}
    # a Secret's files with those names pass the startup check (both entry points run it)
    d = tmp_path
    subprocess.run(["openssl", "req", "-x509", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes",
                    "-days", "1", "-keyout", str(d / "tls.key"), "-out", str(d / "tls.crt"), "-subj", "/CN=gpumon",
                    "-addext", "subjectAltName=DNS:gpumon"], check=True, capture_output=True, timeout=60)
    assert core.check_serve_tls(str(d / os.path.basename(cfg.tls_cert_file)), str(d / os.path.basename(cfg.tls_key_file))) == ""
    # an annotation-driven Prometheus scrapes https too
    ann = _json_patch(ds, ops)["spec"]["template"]["metadata"]["annotations"]
    assert ann["prometheus.io/scheme"] == "https" and ann["prometheus.io/scrape"] == "true"


def test_mutual_tls_overlay_keeps_the_https_probes_working(core, tmp_path):
    """with the overlay's GPUMON_TLS_CLIENT_CA_FILE uncommented, the kubelet's
    httpGet probes (HTTPS, no client certificate, no verification) must still get 200 from /healthz
    and /readyz -- a handshake that required a client certificate failed every probe and restarted
    the pod. /metrics still needs a certificate from the client CA (403 without one)."""
    import http.client
    import ssl
    import subprocess

    (k,) = _docs("deploy/k8s/overlays/tls/kustomization.yaml")
    text = next(p for p in k["patches"] if p["target"]["kind"] == "DaemonSet")["patch"]
    # the mutual-TLS lines as the overlay's comment tells the operator to uncomment them
    lines = text.splitlines()
    i = next(n for n, l in enumerate(lines) if "GPUMON_TLS_CLIENT_CA_FILE" in l)
    for n in range(i - 2, i + 1):
        lines[n] = lines[n].replace("# ", "", 1)
    ops = yaml.safe_load("\n".join(lines))
    ds = next(d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "DaemonSet")
    c = _json_patch(ds, ops)["spec"]["template"]["spec"]["containers"][0]
    env = {e["name"]: e.get("value") for e in c["env"]}
    assert env["GPUMON_TLS_CLIENT_CA_FILE"].endswith("client-ca.crt")
    assert c["livenessProbe"]["httpGet"]["scheme"] == "HTTPS" and c["livenessProbe"]["httpGet"]["path"] == "/healthz"
    files = {}
    for name, cn in (("tls", "gpumon"), ("client-ca", "clients")):
        subprocess.run(["openssl", "req", "-x509", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes",
                        "-days", "1", "-keyout", str(tmp_path / f"{name}.key"), "-out", str(tmp_path / f"{name}.crt"),
                        "-subj", f"/CN={cn}"], check=True, capture_output=True, timeout=60)
        files[name] = str(tmp_path / f"{name}.crt")
    ex = core.Exporter({"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                        "http_threads": 1, "tls_cert_file": files["tls"], "tls_key_file": str(tmp_path / "tls.key"),
                        "tls_client_ca_file": files["client-ca"]})
    assert ex.start() == ""
    try:
        probe = ssl.create_default_context()
        probe.check_hostname = False
        probe.verify_mode = ssl.CERT_NONE  # the kubelet does not verify the serving certificate
        for path, want in ((c["livenessProbe"]["httpGet"]["path"], 200), (c["readinessProbe"]["httpGet"]["path"], 200),
                           ("/metrics", 403)):
            conn = http.client.HTTPSConnection("127.0.0.1", ex.port, context=probe, timeout=5)
            conn.request("GET", path)
            assert conn.getresponse().status == want, path
            conn.close()
    finally:
        ex.stop()


def test_serve_imports_no_oracle_or_grpc():
    """the image's `gpumon serve` (ENTRYPOINT) must not import grpcio / protobuf or
    the Python test oracles -- they live under tests/oracles and are not in the image. The package
    itself no longer contains them."""
    import importlib.util
    import subprocess
    import sys

    for mod in ("gpumon.attribution", "gpumon.ops.pmc", "gpumon.ops.probe"):
        assert importlib.util.find_spec(mod.rsplit(".", 1)[0]) is None or importlib.util.find_spec(mod) is None, mod
    code = r"""
import json, os, signal, sys, threading
from gpumon import cli
threading.Timer(2.0, lambda: os.kill(os.getpid(), signal.SIGTERM)).start()
rc = cli.main(["serve", "--backend", "mock:gpus=1", "--listen", "127.0.0.1:0", "--interval", "0.2",
               "--log-level", "error"])
bad = sorted(m for m in sys.modules if m.split(".")[0] in ("grpc", "oracles") or m.startswith("google.protobuf")
             or m.startswith(("gpumon.attribution", "gpumon.ops.pmc", "gpumon.ops.probe")))
print(json.dumps({"rc": rc, "bad": bad}))
"""
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out == {"rc": 0, "bad": []}, out


def test_dockerfile_installs_no_grpc():
    text = open(os.path.join(ROOT, "deploy", "Dockerfile")).read()
    installs = [l for l in text.splitlines() if "pip3 install" in l]
    assert installs and not any("grpc" in l or "protobuf" in l or "yaml" in l for l in installs), installs
    assert "tests" not in " ".join(l for l in text.splitlines() if l.startswith("COPY")), "oracles stay out of the image"


def test_base_pod_is_unprivileged():
    """the base DaemonSet runs unprivileged -- no privileged flag, no privilege
    escalation, every capability dropped except the two with a named use, and no device node
    mounted (the default exporter opens none: profiles/r3_no_device.md). The reference pod had
    root-equivalent docker.sock access (/root/reference/gpu_monitor.yaml:24-28,38-44)."""
    ds = next(d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "DaemonSet")
    pod = ds["spec"]["template"]["spec"]
    (c,) = pod["containers"]
    sc = c["securityContext"]
    assert sc.get("privileged", False) is False and sc["allowPrivilegeEscalation"] is False
    assert sc["readOnlyRootFilesystem"] is True and sc["seccompProfile"]["type"] == "RuntimeDefault"
    assert sc["capabilities"]["drop"] == ["ALL"]
    # no Kubernetes service-link variables (GPUMON_SERVICE_HOST, ...) in the GPUMON_<KEY> namespace
    assert pod["enableServiceLinks"] is False
    # no DAC_READ_SEARCH in the base (with RuntimeDefault seccomp it unlocks
    # open_by_handle_at); it is the opt-in overlays/fdscan/
    assert sorted(sc["capabilities"].get("add", [])) == ["SYS_NICE", "SYS_PTRACE"]
    assert not pod.get("hostNetwork") and not pod.get("hostIPC")
    mounts = {m["mountPath"] for m in c["volumeMounts"]}
    assert not any(m.startswith("/dev") for m in mounts), mounts
    assert all(not v.get("hostPath", {}).get("path", "").startswith("/dev") for v in pod["volumes"])
    assert {"/var/log/pods", "/var/log/containers"} <= mounts  # socket-free metadata
    assert all(m.get("readOnly") for m in c["volumeMounts"])  # the exporter writes nothing on the host


def test_elevated_rights_only_in_the_ondevice_overlay():
    """PMC device counting and the K1 probe open /dev/kfd: only the ondevice overlay is privileged
    and mounts the device nodes; the docker overlay adds its socket and nothing else."""
    ds = next(d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "DaemonSet")

    def patched(overlay):
        (k,) = _docs(f"deploy/k8s/overlays/{overlay}/kustomization.yaml")
        ops = yaml.safe_load(next(p for p in k["patches"] if p["target"]["kind"] == "DaemonSet")["patch"])
        return _json_patch(ds, ops)["spec"]["template"]["spec"]

    for overlay in ("ondevice", "pmc"):
        pod = patched(overlay)
        c = pod["containers"][0]
        assert c["securityContext"]["privileged"] is True
        assert {"/dev/kfd", "/dev/dri"} <= {m["mountPath"] for m in c["volumeMounts"]}
        vols = {v["name"] for v in pod["volumes"]}
        assert all(m["name"] in vols for m in c["volumeMounts"])
    pod = patched("docker")
    assert pod["containers"][0]["securityContext"].get("privileged", False) is False


def test_service_is_dual_stack_ready():
    """The headless Service asks for both IP families where the cluster has them; the exporter's
    default listen (":9400") answers on both (tests/test_listen.py)."""
    svc = next(d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "Service")
    assert svc["spec"]["ipFamilyPolicy"] == "PreferDualStack" and svc["spec"]["clusterIP"] == "None"


def test_fdscan_overlay_only_adds_dac_read_search():
    """overlays/fdscan/ is the one place CAP_DAC_READ_SEARCH comes back (listing a non-root tenant's
    /proc/<pid>/fd), and its header states the open_by_handle_at trade-off."""
    ds = next(d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "DaemonSet")
    (k,) = _docs("deploy/k8s/overlays/fdscan/kustomization.yaml")
    assert k["resources"] == ["../../"] and [p["target"]["kind"] for p in k["patches"]] == ["DaemonSet"]
    ops = yaml.safe_load(k["patches"][0]["patch"])
    pod = _json_patch(ds, ops)["spec"]["template"]["spec"]
    sc = pod["containers"][0]["securityContext"]
    assert sorted(sc["capabilities"]["add"]) == ["DAC_READ_SEARCH", "SYS_NICE", "SYS_PTRACE"]
    base = ds["spec"]["template"]["spec"]["containers"][0]["securityContext"]
    assert {k2: v for k2, v in sc.items() if k2 != "capabilities"} == {k2: v for k2, v in base.items() if k2 != "capabilities"}
    text = open(os.path.join(ROOT, "deploy/k8s/overlays/fdscan/kustomization.yaml")).read()
    assert "open_by_handle_at" in text and "seccomp" in text


def test_nonroot_overlay():
    """A strictly non-root pod: no capabilities, runAsNonRoot, no kubelet / CRI socket (they accept
    root only), pod metadata from the kubelet's log tree (csrc/core/kubelet_files.h)."""
    from gpumon.config import Config

    (k,) = _docs("deploy/k8s/overlays/nonroot/kustomization.yaml")
    assert k["resources"] == ["../../"]
    cfg_patch = next(p for p in k["patches"] if p["target"]["kind"] == "ConfigMap")
    c = Config().apply_dict(yaml.safe_load(yaml.safe_load(cfg_patch["patch"])[0]["value"])["gpumon"])
    assert c.pod_log_root == "/var/log" and c.cri_socket == "none" and c.pod_resources_socket == ""
    assert c.rt_priority == 0 and c.http_rt_priority == 0
    ds = next(d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "DaemonSet")
    ops = yaml.safe_load(next(p for p in k["patches"] if p["target"]["kind"] == "DaemonSet")["patch"])
    ctr = _json_patch(ds, ops)["spec"]["template"]["spec"]["containers"][0]
    sc = ctr["securityContext"]
    assert sc["runAsNonRoot"] is True and sc["runAsUser"] != 0 and sc["capabilities"] == {"drop": ["ALL"]}
    assert sc["allowPrivilegeEscalation"] is False and not sc.get("privileged")
    assert {"/var/log/pods", "/var/log/containers"} <= {m["mountPath"] for m in ctr["volumeMounts"]}


def test_overlay_configs_are_valid_for_the_native_binary(tmp_path):
    """Every overlay's ConfigMap is accepted by bin/gpumon-exporter --config (the Python-free
    entrypoint reads the same keys)."""
    import subprocess

    from conftest import make_locked

    make_locked("core")
    base = next(d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "ConfigMap")
    values = {"base": base["data"]["config.yaml"]}
    for overlay in ("ondevice", "pmc", "docker", "nonroot", "stress"):
        (k,) = _docs(f"deploy/k8s/overlays/{overlay}/kustomization.yaml")
        values[overlay] = yaml.safe_load(next(p for p in k["patches"]
                                              if p["target"]["kind"] == "ConfigMap")["patch"])[0]["value"]
    for name, value in values.items():
        f = tmp_path / f"{name}.yaml"
        f.write_text(value)
        r = subprocess.run([os.path.join(ROOT, "bin", "gpumon-exporter"), "--config", str(f), "--print-config"],
                           capture_output=True, text=True, timeout=30)
        assert r.returncode == 0, (name, r.stderr[-1000:])
        # the native binary is the image's entrypoint: no key it would ignore, no unknown key
        assert "unknown" not in r.stderr.lower() and "not used" not in r.stderr, (name, r.stderr[-1000:])
        assert json.loads(r.stdout)["listen"] == ":9400", name


def test_stress_overlay_is_10hz_end_to_end():
    """BASELINE.json's stress config (10 Hz sampling, Prometheus scraping at 10 Hz): the overlay
    sets both, and its CPU request covers the measured 8-device 10 Hz cost with headroom (91
    millicores at 200 gzip scrapes/s in the 8x rehearsal, an upper bound: profiles/r5_cpu_8dev.md)."""
    from gpumon.config import Config

    (k,) = _docs("deploy/k8s/overlays/stress/kustomization.yaml")
    assert k["resources"] == ["../../"]
    cfg_patch = next(p for p in k["patches"] if p["target"]["kind"] == "ConfigMap")
    c = Config().apply_dict(yaml.safe_load(yaml.safe_load(cfg_patch["patch"])[0]["value"])["gpumon"])
    assert c.interval == pytest.approx(0.1)
    base = next(d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "ConfigMap")
    b = Config().apply_dict(yaml.safe_load(base["data"]["config.yaml"])["gpumon"])
    for key in ("pod_resources_socket", "cri_socket", "pod_log_root", "rt_priority", "http_rt_priority", "control_plane",
                "enable_pmc", "enable_probe"):
        assert getattr(c, key) == getattr(b, key), key  # only the rate differs from the base
    sm = _docs("deploy/k8s/gpumon-servicemonitor.yaml")[0]
    ops = yaml.safe_load(next(p for p in k["patches"] if p["target"]["kind"] == "ServiceMonitor")["patch"])
    ep = _json_patch(sm, ops)["spec"]["endpoints"][0]
    assert ep["interval"] == "100ms" and ep["scrapeTimeout"] == "90ms"
    ds = next(d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "DaemonSet")
    ops = yaml.safe_load(next(p for p in k["patches"] if p["target"]["kind"] == "DaemonSet")["patch"])
    ctr = _json_patch(ds, ops)["spec"]["template"]["spec"]["containers"][0]
    assert int(ctr["resources"]["requests"]["cpu"].rstrip("m")) >= 1.3 * 91
    assert not ctr["securityContext"].get("privileged")


def test_systemd_unit_for_bare_metal_nodes(tmp_path):
    """deploy/systemd/: the same native binary and config format without Kubernetes. The unit's
    command line and config parse (no ignored keys) identically in both entry points, it grants the
    DaemonSet's two capabilities and nothing else, and exit status 2 (a configuration error) is not
    restarted in a loop."""
    import configparser
    import json
    import shlex
    import subprocess

    from gpumon.config import Config, load_yaml

    unit = configparser.ConfigParser(strict=False, interpolation=None)
    unit.optionxform = str
    unit.read(os.path.join(ROOT, "deploy/systemd/gpumon-exporter.service"))
    svc = unit["Service"]
    argv = shlex.split(svc["ExecStart"])
    assert argv[0].endswith("/gpumon-exporter") and argv[1:] == ["--config", "/etc/gpumon/config.yaml"]
    assert svc["RestartPreventExitStatus"] == "2" and svc["ExecReload"].endswith("-HUP $MAINPID")
    ds = next(d for d in _docs("deploy/k8s/gpumon-daemonset.yaml") if d["kind"] == "DaemonSet")
    caps = ds["spec"]["template"]["spec"]["containers"][0]["securityContext"]["capabilities"]["add"]
    assert sorted(svc["CapabilityBoundingSet"].split()) == sorted("CAP_" + c for c in caps)
    cfg_path = os.path.join(ROOT, "deploy/systemd/config.yaml")
    r = subprocess.run([os.path.join(ROOT, "bin", "gpumon-exporter"), "--config", cfg_path, "--print-config"],
                       capture_output=True, text=True, timeout=30)
    assert r.returncode == 0 and "ignored" not in r.stderr, r.stderr
    native = json.loads(r.stdout)
    py = Config().apply_dict(load_yaml(cfg_path))
    assert native["include_host_processes"] is True and py.include_host_processes is True
    assert native["cri_socket"] == py.cri_socket == "none" and native["pod_resources_socket"] == py.pod_resources_socket == ""
