"""`gpumon doctor` (gpumon/doctor.py): the node-prerequisite report, against the mock backend and
the fake kubelet. The reference's only self-check was commandexists('docker'/'nvidia-smi')
(/root/reference/gpu.py:28-33,260)."""

import json
import os
import socket
import subprocess
import sys

import grpc
import pytest

from oracles.attribution.fake_kubelet import FakeKubelet
from gpumon.config import Config
from gpumon import doctor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _by_name(checks):
    return {c: (s, d) for c, s, d in checks}


def test_doctor_reports_sockets_and_plugins():
    d = f"/tmp/gpumon-doc-{os.getpid()}"
    os.makedirs(d, exist_ok=True)
    with FakeKubelet(podres_socket=f"{d}/kubelet.sock", cri_socket=f"{d}/cri.sock") as k:
        cfg = Config(backend="mock:gpus=2", control_plane="native", pod_resources_socket=k.podres_socket,
                     cri_socket=k.cri_socket, log_level="error")
        checks = _by_name(doctor.run(cfg, wait_s=5))
    assert checks["device backend"][0] == "ok" and "2 GPU(s)" in checks["device backend"][1]
    assert checks["kubelet PodResources"][0] == "ok" and checks["CRI runtime"][0] == "ok"
    assert checks["sysfs fast path"][0] == "skip"  # mock backend
    assert checks["on-device plugins"][0] == "ok"
    assert checks["rt_priority / http_rt_priority"][0] in ("ok", "warn")
    assert checks["other uids' fd tables"][0] in ("ok", "warn", "skip")
    assert checks["file descriptor limit"][0] in ("ok", "warn")


def test_doctor_names_the_grpc_status_of_a_refusing_kubelet():
    d = f"/tmp/gpumon-doc2-{os.getpid()}"
    os.makedirs(d, exist_ok=True)
    with FakeKubelet(podres_socket=f"{d}/kubelet.sock") as k:
        k.podres_error = (grpc.StatusCode.PERMISSION_DENIED, "socket is root-only")
        cfg = Config(backend="mock:gpus=1", control_plane="native", pod_resources_socket=k.podres_socket,
                     cri_socket="", log_level="error")
        checks = _by_name(doctor.run(cfg, wait_s=5))
    s, detail = checks["kubelet PodResources"]
    assert s == "warn" and "grpc-status 7" in detail and "idle-allocation" in detail


def test_doctor_cli_json_and_exit_status():
    r = subprocess.run([sys.executable, "-m", "gpumon", "doctor", "--backend", "mock:gpus=1", "--format", "json",
                        "--control-plane", "off"], capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = {x["check"]: x for x in json.loads(r.stdout)}
    assert rows["device backend"]["status"] == "ok" and rows["listen address"]["status"] in ("ok", "warn")
    # a backend that cannot come up is the one failing (exit 1) check
    r = subprocess.run([sys.executable, "-m", "gpumon", "doctor", "--backend", "rocm_smi", "--format", "json",
                        "--control-plane", "off"], capture_output=True, text=True, timeout=120, cwd=ROOT,
                       env=dict(os.environ, LD_LIBRARY_PATH="/nonexistent"))
    rows = {x["check"]: x for x in json.loads(r.stdout)}
    assert r.returncode == 1 and rows["device backend"]["status"] == "fail", (r.returncode, rows)


def test_doctor_runs_the_ondevice_samplers_once():
    from conftest import make_locked

    make_locked("fakes")
    cfg = Config(backend="mock:gpus=1", control_plane="off", log_level="error",
                 plugin_dir=os.path.join(ROOT, "build", "fakes", "ondevice"))
    checks = _by_name(doctor.run(cfg, ondevice_check=True, wait_s=0.5))
    assert checks["PMC device counting"][0] == "ok", checks
    assert checks["K1 probe"][0] == "ok", checks
    assert checks["on-device helper memory"][0] == "ok"


def test_doctor_checks_the_docker_socket_when_configured():
    from test_docker import CID_PLAIN, FakeDocker, _container

    sock = f"/tmp/gpumon-doc3-{os.getpid()}.sock"
    with FakeDocker(sock, [_container(CID_PLAIN, "bench", {})]):
        cfg = Config(backend="mock:gpus=1", control_plane="native", pod_resources_socket="", cri_socket="",
                     docker_socket=sock, log_level="error")
        s, detail = _by_name(doctor.run(cfg, wait_s=1))["Docker Engine"]
    assert s == "ok" and sock in detail
    with FakeDocker(sock, [], status=403):
        cfg = Config(backend="mock:gpus=1", control_plane="native", pod_resources_socket="", cri_socket="",
                     docker_socket=sock, log_level="error")
        s, detail = _by_name(doctor.run(cfg, wait_s=1))["Docker Engine"]
    assert s == "warn" and "http-status 403" in detail
    s, _ = _by_name(doctor.run(Config(backend="mock:gpus=1", control_plane="native", pod_resources_socket="",
                                      cri_socket="", log_level="error"), wait_s=1))["Docker Engine"]
    assert s == "skip"  # never autodetected


def test_doctor_checks_the_kubelet_files_when_configured(tmp_path):
    """Non-root deployments name pods from the kubelet's log tree: the doctor says whether it (and
    the device-plugin checkpoint) could be read."""
    (tmp_path / "log" / "pods").mkdir(parents=True)
    (tmp_path / "log" / "containers").mkdir()
    cfg = Config(backend="mock:gpus=1", control_plane="native", pod_resources_socket="", cri_socket="none",
                 pod_log_root=str(tmp_path / "log"), device_checkpoint=str(tmp_path / "missing"), log_level="error")
    checks = _by_name(doctor.run(cfg, wait_s=1))
    assert checks["kubelet log tree"][0] == "ok", checks["kubelet log tree"]
    assert checks["device-plugin checkpoint"][0] == "warn" and "unreadable" in checks["device-plugin checkpoint"][1]
    cfg = Config(backend="mock:gpus=1", control_plane="native", pod_resources_socket="", cri_socket="none",
                 log_level="error")
    checks = _by_name(doctor.run(cfg, wait_s=1))
    assert checks["kubelet log tree"][0] == "skip"


def _fake_gpu_metrics(path, period_s, stop):
    """A v1.8-shaped table file whose firmware_timestamp (offset 288) a thread bumps every period."""
    import struct
    import threading

    buf = bytearray(3872)
    struct.pack_into("<HBB", buf, 0, 3872, 1, 8)
    path.write_bytes(bytes(buf))

    def bump():
        fw = 1
        with open(path, "r+b") as fh:
            while not stop.is_set():
                fw += int(period_s * 1e8)
                fh.seek(288)
                fh.write(struct.pack("<Q", fw))
                fh.flush()
                stop.wait(period_s)

    t = threading.Thread(target=bump, daemon=True)
    t.start()
    return t


def test_doctor_firmware_table_cadence_against_the_interval(tmp_path):
    """The SMU rewrites gpu_metrics every 20 ms on MI355X: doctor reports the period it measures and
    warns when the configured interval is shorter (those samples repeat a table)."""
    import re
    import threading

    from gpumon.doctor import OK, WARN, firmware_table_check

    stop = threading.Event()
    f = tmp_path / "gpu_metrics"
    t = _fake_gpu_metrics(f, 0.02, stop)
    try:
        st, detail = firmware_table_check(str(f), 1.0, 3.0, seconds=0.3)
        assert st == OK, detail
        period = float(re.search(r"every ([0-9.]+) ms", detail).group(1))
        assert 15 <= period <= 35, detail
        st, detail = firmware_table_check(str(f), 0.005, 3.0, seconds=0.3)
        assert st == WARN and "interval 5 ms is shorter" in detail, detail
    finally:
        stop.set()
        t.join()


def test_doctor_fd_limit_matches_the_server_cap():
    """The doctor's connection cap is the one HttpServer::start derives from RLIMIT_NOFILE."""
    from gpumon.doctor import OK, WARN, fd_limit_check

    assert fd_limit_check(2, limit=1048576) == (OK, "RLIMIT_NOFILE 1048576: 4096 connections per HTTP loop (2 loop(s))")
    st, detail = fd_limit_check(2, limit=1024)
    assert st == OK and "384 connections per HTTP loop" in detail  # (1024 - 256) / 2
    st, detail = fd_limit_check(2, limit=64)
    assert st == WARN and "16 connections per HTTP loop" in detail  # 64 / 2 / 2


def test_doctor_cap_formula_is_the_servers(core):
    """doctor.fd_limit_cap and HttpServer::start compute the same cap at this process's limit."""
    from gpumon.doctor import fd_limit_cap

    for threads in (1, 2, 3):
        ex = core.Exporter({"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                            "http_threads": threads})
        ex.start()
        try:
            assert ex.self_stats()["http_max_conns"] == threads * fd_limit_cap(threads)
        finally:
            ex.stop()


@pytest.mark.parametrize("entry", ["native", "python"])
def test_serve_raises_the_soft_fd_limit_to_the_hard_one(entry):
    """Container runtimes often start a pod at a soft nofile limit of 1024 under a high hard limit:
    both entry points raise the soft limit, so the connection cap (gpumon_http_max_connections)
    comes from the hard one."""
    import os
    import resource
    import subprocess
    import sys
    import time
    import urllib.request

    from gpumon.doctor import fd_limit_cap
    from gpumon.export import promtext

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hard = resource.getrlimit(resource.RLIMIT_NOFILE)[1]
    if hard != resource.RLIM_INFINITY and hard < 2048:
        pytest.skip(f"hard nofile limit {hard}: nothing to raise to")
    hard = 4096  # a definite value under this process's hard limit

    def limits():
        resource.setrlimit(resource.RLIMIT_NOFILE, (512, hard))

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = ([os.path.join(root, "bin", "gpumon-exporter")] if entry == "native"
           else [sys.executable, "-m", "gpumon", "serve", "--control-plane", "off"])
    cmd += ["--backend", "mock:gpus=1", "--interval", "0.2", "--listen", f"127.0.0.1:{port}", "--http-threads", "2"]
    p = subprocess.Popen(cmd, cwd=root, env=dict(os.environ, PYTHONPATH=root), stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL, preexec_fn=limits)
    try:
        body = None
        deadline = time.time() + 30
        while time.time() < deadline and body is None:
            try:
                body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=2).read().decode()
            except OSError:
                time.sleep(0.1)
        assert body is not None
        with open(f"/proc/{p.pid}/limits") as fh:
            row = next(l for l in fh if l.startswith("Max open files")).split()
        assert row[3:5] == [str(hard), str(hard)], row
        fam = promtext.parse(body)
        assert promtext.one(fam, "gpumon_http_max_connections") == 2 * fd_limit_cap(2, limit=hard)
    finally:
        p.terminate()
        p.wait(10)


def test_doctor_checks_the_listen_address():
    import socket

    assert doctor.listen_check("127.0.0.1:0")[0] == "ok"
    assert doctor.listen_check("nope")[0] == "fail"
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    s.listen(1)
    port = s.getsockname()[1]
    try:
        st, detail = doctor.listen_check(f"127.0.0.1:{port}")
        assert st == "warn" and "in use" in detail and "EADDRINUSE" in detail
    finally:
        s.close()
    st, detail = doctor.listen_check(f"127.0.0.1:{port}")
    assert st == "ok" and "free" in detail and "IPv4 only" in detail
    st, detail = doctor.listen_check(":0")
    assert st == "ok" and ("dual-stack" in detail or "IPv4 only" in detail)


def test_doctor_checks_the_influx_push(tmp_path):
    """The push's startup check (named failure: the exporter would refuse to start) and a /ping on
    the same host over the same transport: an answering InfluxDB, a closed port, an https URL
    whose certificate does not verify."""
    import http.server
    import threading

    class Ping(http.server.BaseHTTPRequestHandler):
        def do_GET(self):  # noqa: N802
            self.send_response(204 if self.path == "/ping" else 404)
            self.send_header("Content-Length", "0")
            self.end_headers()

        def log_message(self, *a):
            pass

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), Ping)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        ok = doctor.influx_check(Config(influx_url=f"http://u:pw@127.0.0.1:{srv.server_port}/write?db=k8s"))
        assert ok[0] == "ok" and "/ping answered 204" in ok[1] and "pw" not in ok[1]
    finally:
        srv.shutdown()
    bad = doctor.influx_check(Config(influx_url="ftp://influx/write"))
    assert bad[0] == "fail" and "unsupported scheme" in bad[1]
    down = doctor.influx_check(Config(influx_url="http://127.0.0.1:9/write"))
    assert down[0] == "warn" and "connect" in down[1]
    checks = _by_name(doctor.run(Config(backend="mock:gpus=1", control_plane="off", log_level="error",
                                        influx_url="ftp://influx/write"), wait_s=0.2))
    assert checks["Influx push"][0] == "fail" and checks["device backend"][0] == "ok"


def test_doctor_reports_the_metrics_certificate(tmp_path):
    """/metrics over HTTPS: the doctor says whether the certificate loads and how long it is valid
    (warn under 7 days, fail once expired or unloadable)."""
    import time

    from gpumon.doctor import FAIL, OK, WARN, serve_tls_check

    subprocess.run(["openssl", "req", "-x509", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes",
                    "-days", "30", "-keyout", str(tmp_path / "k.pem"), "-out", str(tmp_path / "c.pem"), "-subj",
                    "/CN=gpumon"], check=True, capture_output=True, timeout=60)
    cfg = Config(tls_cert_file=str(tmp_path / "c.pem"), tls_key_file=str(tmp_path / "k.pem"))
    st, detail = serve_tls_check(cfg)
    assert st == OK and "valid until" in detail and ("(30 days)" in detail or "(29 days)" in detail), detail
    st, detail = serve_tls_check(cfg, now=time.time() + 26 * 86400)
    assert st == WARN and "expires" in detail, detail
    st, detail = serve_tls_check(cfg, now=time.time() + 31 * 86400)
    assert st == FAIL and "EXPIRED" in detail, detail
    st, detail = serve_tls_check(Config(tls_cert_file=str(tmp_path / "c.pem")))
    assert st == FAIL and "go together" in detail
    checks = _by_name(doctor.run(Config(backend="mock:gpus=1", control_plane="off", log_level="error",
                                        tls_cert_file=str(tmp_path / "c.pem"), tls_key_file=str(tmp_path / "k.pem")),
                                 wait_s=0.5))
    assert checks["/metrics TLS certificate"][0] == OK


def test_doctor_checks_the_kfd_queue_lists(tmp_path):
    """The peer-context rule reads KFD's per-process queue lists; the doctor says whether it can."""
    from gpumon.doctor import OK, SKIP, WARN, kfd_queue_check

    kfd = tmp_path / "proc"
    assert kfd_queue_check(str(kfd))[0] == SKIP  # no KFD at all
    kfd.mkdir()
    assert kfd_queue_check(str(kfd))[0] == SKIP  # no process to try
    for pid, nq in ((100, 2), (200, 0)):
        (kfd / str(pid) / "queues").mkdir(parents=True)
        for q in range(nq):
            (kfd / str(pid) / "queues" / str(q)).mkdir()
    st, detail = kfd_queue_check(str(kfd))
    assert st == OK and "2/2" in detail and "2 queue(s)" in detail
    # unreadable lists (an older kernel without queues/, or no rights): a file stands in here, since
    # root would read a mode-000 directory anyway
    import shutil

    for pid in (100, 200):
        shutil.rmtree(kfd / str(pid) / "queues")
        (kfd / str(pid) / "queues").write_text("")
    st, detail = kfd_queue_check(str(kfd))
    assert st == WARN and "peer_context_max_vram_mib" in detail
