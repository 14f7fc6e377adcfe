"""Host-side sanitizer runs of the native exporter (SURVEY.md §5 race detection): ASan+UBSan and
TSan builds of bin/gpumon-exporter under concurrent scrapes while the sampler ticks at 100 Hz and
snapshots are swapped. GPU sanitizers are not available on this pool; these cover the C++ core."""

import os
import re
import signal
import socket
import subprocess
import threading
import time
import urllib.error
import urllib.request

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _reports(stderr):
    """Sanitizer report lines (ASan, UBSan, TSan, LeakSanitizer) in a run's stderr."""
    return [l for l in stderr.splitlines() if "ERROR: AddressSanitizer" in l or "runtime error:" in l
            or "WARNING: ThreadSanitizer" in l or "ERROR: LeakSanitizer" in l]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(binary, env_extra, extra_args=(), min_s=0.0, ctx=None, port=None, token=None, until=None):
    """ctx: an ssl.SSLContext to scrape over HTTPS (the exporter started with --tls-cert-file);
    token: the bearer token to scrape with (--http-auth-token-file); until: after min_s, keep the
    exporter running (up to 30 s more) until this returns true -- a sanitized build on a loaded host
    does in 2 s what a plain one does in a fraction of it."""
    port = port or _free_port()
    base = f"https://localhost:{port}" if ctx else f"http://127.0.0.1:{port}"
    t_start = time.time()
    env = dict(os.environ, **env_extra)
    p = subprocess.Popen([binary, "--backend", "mock:gpus=4", "--interval", "0.01", "--listen", f"127.0.0.1:{port}",
                          "--sample-threads", "2", "--http-threads", "2", "--log-level", "error", *extra_args],
                         stderr=subprocess.PIPE, stdout=subprocess.DEVNULL, env=env, text=True)
    try:
        deadline = time.time() + 30
        while time.time() < deadline:
            try:
                urllib.request.urlopen(f"{base}/healthz", timeout=1, context=ctx).read()
                break
            except OSError:
                time.sleep(0.1)
        errors = []

        def hammer(query):
            for _ in range(60):
                try:
                    hdr = {"Accept-Encoding": "gzip", **({"Authorization": f"Bearer {token}"} if token else {})}
                    req = urllib.request.Request(f"{base}/metrics{query}", headers=hdr)
                    urllib.request.urlopen(req, timeout=5, context=ctx).read()
                except Exception as e:  # noqa: BLE001
                    errors.append(e)

        # plain scrapes and per-request family filters (the per-snapshot filter cache) side by side
        ts = [threading.Thread(target=hammer, args=(q,))
              for q in ("", "", "?exclude=gpu_xcd_*", "?include=node_gpu_*,gpu_up")]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errors, errors[:3]
        time.sleep(max(0.0, t_start + min_s - time.time()))  # background pollers get their refreshes
        t_until = time.time() + 30
        while until is not None and not until() and time.time() < t_until:
            time.sleep(0.1)
    finally:
        p.send_signal(signal.SIGTERM)
        _, err = p.communicate(timeout=60)
    return p.returncode, err


# the on-device sampler threads (csrc/core/ondevice.cpp) over the fake plugins, plus a RAS refresh
# every tick: PMC / probe / RAS state crosses threads into set_extra() and the renderer
ONDEVICE = ("--pmc", "--probe", "--plugin-dir", os.path.join(ROOT, "build", "fakes", "ondevice"), "--ras-every", "1")


@pytest.mark.slow
@pytest.mark.parametrize("extra", [(), ONDEVICE], ids=["core", "ondevice"])
@pytest.mark.parametrize("target,binary,env", [
    ("asan", "bin/gpumon-exporter-asan", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                                          "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}),
    ("tsan", "bin/gpumon-exporter-tsan", {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}),
])
def test_sanitized_exporter_under_concurrent_scrapes(target, binary, env, extra):
    from conftest import make_locked

    r = make_locked(target, *(["fakes"] if extra else []), jobs=8)
    assert r.returncode == 0, r.stderr[-2000:]
    rc, err = _run(os.path.join(ROOT, binary), dict(env, GPUMON_FAKE_AGENTS="4"), extra)
    bad = _reports(err)
    assert not bad, err[-4000:]
    assert rc == 0, err[-2000:]


@pytest.mark.slow
@pytest.mark.parametrize("target,binary,env", [
    ("asan", "bin/gpumon-exporter-asan", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                                          "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}),
    ("tsan", "bin/gpumon-exporter-tsan", {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}),
])
def test_sanitized_exporter_survives_helper_kills(target, binary, env):
    """The on-device helper SIGKILLed three times while the PMC and probe threads both use it: the
    respawn path (one sampler respawns, the other waits on it; PMC re-init before probe ops) runs
    under ASan/UBSan and TSan without a report, and the exporter keeps serving."""
    from conftest import make_locked

    make_locked(target, "fakes", jobs=8)
    port = _free_port()
    e = dict(os.environ, GPUMON_FAKE_AGENTS="2", **env)
    p = subprocess.Popen([os.path.join(ROOT, binary), "--backend", "mock:gpus=2", "--interval", "0.02", "--listen",
                          f"127.0.0.1:{port}", "--log-level", "error", "--pmc", "--probe", "--probe-every", "1",
                          "--plugin-dir", os.path.join(ROOT, "build", "fakes", "ondevice")],
                         stderr=subprocess.PIPE, stdout=subprocess.DEVNULL, env=dict(e, GPUMON_HELPER_RETRY="0.05"),
                         text=True)
    try:
        def helpers():
            out = []
            for q in os.listdir("/proc"):
                if q.isdigit():
                    try:
                        if open(f"/proc/{q}/comm").read().strip() == "gpumon-ondevice" and \
                                int(open(f"/proc/{q}/stat").read().rsplit(")", 1)[1].split()[1]) == p.pid:
                            out.append(int(q))
                    except (OSError, ValueError, IndexError):
                        pass
            return out

        deadline = time.time() + 150  # a sanitized helper's respawn + PMC init on a loaded host: tens of s
        kills = 0
        while kills < 3 and time.time() < deadline:
            hs = helpers()
            if hs:
                os.kill(hs[0], signal.SIGKILL)
                kills += 1
                time.sleep(0.3)
            else:
                time.sleep(0.05)
        assert kills == 3
        time.sleep(1.0)
        assert p.poll() is None
        body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
        restarts = float(re.search(r"^gpumon_ondevice_helper_restarts_total\{[^}]*\} (\S+)$", body, re.M).group(1))
        assert restarts >= 2, restarts
    finally:
        p.send_signal(signal.SIGTERM)
        _, err = p.communicate(timeout=60)
    bad = _reports(err)
    assert not bad, err[-4000:]


@pytest.mark.slow
@pytest.mark.parametrize("target,binary,env", [
    ("asan", "bin/gpumon-exporter-asan", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                                          "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}),
    ("tsan", "bin/gpumon-exporter-tsan", {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}),
])
def test_sanitized_docker_poller_on_mutated_listings(target, binary, env):
    """The Docker Engine poller (csrc/core/docker_lite.cpp) refreshing every 0.5 s against a fake
    daemon whose every answer is a random mutation of a realistic listing (truncations, byte flips,
    duplicated spans) while scrapes run: no ASan/UBSan/TSan report and the exporter keeps serving."""
    import json
    import random

    from conftest import make_locked
    from test_docker import CID_K8S, CID_PLAIN, K8S_LABELS, FakeDocker, _container

    make_locked(target, jobs=8)
    good = json.dumps([_container(CID_K8S, "k8s_nb", K8S_LABELS),
                       _container(CID_PLAIN, "b\u00f6b", {"mlgpu": "mlgpu", "emoji": "\U0001F600"})]).encode()
    rng = random.Random(7)
    served = []

    def mutate():
        b = bytearray(good)
        for _ in range(rng.randint(0, 6)):
            op, i = rng.randrange(3), rng.randrange(len(b))
            if op == 0:
                b[i] = rng.randrange(256)
            elif op == 1:
                del b[i:i + rng.randint(1, 40)]
            else:
                b[i:i] = b[i:i + rng.randint(1, 40)]
        served.append(len(b))
        return bytes(b)

    sock = f"/tmp/gpumon-docker-san-{target}-{os.getpid()}.sock"
    with FakeDocker(sock, mutate):
        rc, err = _run(os.path.join(ROOT, binary), dict(env, GPUMON_METADATA_REFRESH="0.5"), ("--docker", sock),
                       min_s=4.0)
    bad = _reports(err)
    assert not bad, err[-4000:]
    assert rc == 0, err[-2000:]
    assert len(served) >= 4, served


@pytest.mark.slow
@pytest.mark.parametrize("target,binary,env", [
    ("asan", "bin/gpumon-exporter-asan", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                                          "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}),
    ("tsan", "bin/gpumon-exporter-tsan", {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}),
])
def test_sanitized_sharing_subsamples_and_link_map(target, binary, env, tmp_path):
    """The round-3 threads and state: three processes per GPU (sharing state, arrivals), the device
    workers' between-tick KFD scans racing the per-device process-list threads, the xGMI slot map
    refreshed every tick over a rotated entry order, and the kubelet-files poller (log tree and a
    device-plugin checkpoint) -- under ASan/UBSan and TSan while scrapes run."""
    import json

    from conftest import make_locked

    make_locked(target, jobs=8)
    logs = tmp_path / "log"
    (logs / "pods" / "ns_p-0_uid-1" / "c").mkdir(parents=True)
    (logs / "containers").mkdir()
    os.symlink("/var/log/pods/ns_p-0_uid-1/c/0.log", logs / "containers" / f"p-0_ns_c-{'a' * 64}.log")
    ckpt = tmp_path / "ckpt"
    ckpt.write_text(json.dumps({"Data": {"PodDeviceEntries": [
        {"PodUID": "uid-1", "ContainerName": "c", "ResourceName": "amd.com/gpu", "DeviceIDs": {"0": ["x"]},
         "AllocResp": ""}]}, "Checksum": 1}))
    rc, err = _run(os.path.join(ROOT, binary), dict(env, GPUMON_LINK_EVERY="1", GPUMON_OCC_SAMPLES="20"),
                   ("--backend", "mock:gpus=4,procs=3,link_order=rotate", "--interval", "0.1",
                    "--pod-logs", str(logs), "--device-checkpoint", str(ckpt)), min_s=3.0)
    bad = _reports(err)
    assert not bad, err[-4000:]
    assert rc == 0, err[-2000:]


class _GarbageH2:
    """A unix-socket 'kubelet' that answers every connection with a seeded random mix of valid
    and mangled HTTP/2 frames (the frame kinds grpc_lite.cpp handles, with bad lengths, padding and
    flags), then hangs up: the native gRPC client's parser under the sanitizers."""

    def __init__(self, path, seed=11):
        import random
        import struct

        self.path, self.rng, self.struct, self.n = path, random.Random(seed), struct, 0
        if os.path.exists(path):
            os.unlink(path)
        self.srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.srv.bind(path)
        self.srv.listen(8)
        self.srv.settimeout(0.2)
        self.stop = threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _frame(self):
        r, st = self.rng, self.struct
        typ = r.choice([0, 1, 3, 4, 6, 7, 8, 9, 0x42])
        flags = r.choice([0, 1, 4, 5, 8, 0x20, 0x2d, 0xff])
        payload = bytes(r.randrange(256) for _ in range(r.choice([0, 1, 2, 5, 9, 40])))
        if typ in (0, 1) and r.random() < 0.5:  # a well-formed gRPC message / header block
            payload = b"\x00" + st.pack(">I", 3) + b"\x0a\x01a" if typ == 0 else b"\x00\x07:status\x03200"
        n = len(payload) if r.random() < 0.8 else r.randrange(1 << 24)
        return st.pack(">I", n)[1:] + bytes([typ, flags]) + st.pack(">I", r.choice([0, 1, 3])) + payload

    def _run(self):
        while not self.stop.is_set():
            try:
                conn, _ = self.srv.accept()
            except OSError:
                continue
            self.n += 1
            try:
                conn.settimeout(0.5)
                conn.recv(4096)
                conn.sendall(b"".join(self._frame() for _ in range(self.rng.randint(1, 8))))
            except OSError:
                pass
            finally:
                conn.close()

    def close(self):
        self.stop.set()
        self.t.join(5)
        self.srv.close()
        os.unlink(self.path)


@pytest.mark.slow
@pytest.mark.parametrize("target,binary,env", [
    ("asan", "bin/gpumon-exporter-asan", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                                          "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}),
    ("tsan", "bin/gpumon-exporter-tsan", {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}),
])
def test_sanitized_failure_paths(target, binary, env):
    """Round-4 failure paths: a start that fails at the listen address (backend and device workers
    already up: the leak checker sees whatever is not taken down), process lists that fail every
    3rd call (the held list crossing threads), a PodResources / CRI peer that answers mangled
    HTTP/2, and an Influx push that cannot connect (requeue + backoff) -- with scrapes running, no
    sanitizer report."""
    from conftest import make_locked

    make_locked(target, jobs=8)
    exe = os.path.join(ROOT, binary)
    r = subprocess.run([exe, "--backend", "mock:gpus=4", "--sample-threads", "2", "--listen", "not-an-address:1",
                        "--log-level", "error"], capture_output=True, text=True, timeout=60, env=dict(os.environ, **env))
    bad = _reports(r.stderr)
    assert not bad, r.stderr[-4000:]
    assert r.returncode not in (0, -6, -11, 134, 139), r.stderr[-2000:]
    sock = f"/tmp/gpumon-h2-san-{target}-{os.getpid()}.sock"
    peer = _GarbageH2(sock)
    try:
        # plus an Influx push to a port nothing listens on: the pusher's requeue + backoff path
        rc, err = _run(exe, dict(env, GPUMON_METADATA_REFRESH="0.3", GPUMON_INFLUX_TIMEOUT_S="0.2"),
                       ("--backend", "mock:gpus=4,procs=3,procs_fail_every=3", "--interval", "0.05",
                        "--pod-resources", sock, "--cri", sock, "--influx-url", "http://127.0.0.1:9/write"),
                       min_s=3.0)
    finally:
        peer.close()
    bad = _reports(err)
    assert not bad, err[-4000:]
    assert rc == 0, err[-2000:]
    assert peer.n >= 4, peer.n


@pytest.mark.slow
def test_tsan_readyz_while_the_backend_keeps_failing_to_initialise():
    """/readyz reports the backend's init error while the sampler re-tries the init every tick:
    the error string is shared between the two threads (err_mu_), which TSan checks here."""
    from conftest import make_locked

    make_locked("tsan", jobs=8)
    port = _free_port()
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1",
               GPUMON_AMDSMI_LIB="/nonexistent/libamd_smi.so", GPUMON_INIT_RETRY_S="0.002")
    p = subprocess.Popen([os.path.join(ROOT, "bin/gpumon-exporter-tsan"), "--backend", "amdsmi", "--interval", "0.005",
                          "--listen", f"127.0.0.1:{port}", "--http-threads", "2", "--log-level", "error"],
                         stderr=subprocess.PIPE, stdout=subprocess.DEVNULL, env=env, text=True)
    codes = []
    try:
        deadline = time.time() + 30
        while time.time() < deadline:
            try:
                urllib.request.urlopen(f"http://127.0.0.1:{port}/healthz", timeout=1).read()
                break
            except OSError:
                time.sleep(0.1)

        def hammer():
            for _ in range(150):
                try:
                    urllib.request.urlopen(f"http://127.0.0.1:{port}/readyz", timeout=5)
                    codes.append(200)
                except urllib.error.HTTPError as e:
                    codes.append(e.code)
                    body = e.read().decode()
                    assert body.startswith("not ready: "), body

        ts = [threading.Thread(target=hammer) for _ in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    finally:
        p.send_signal(signal.SIGTERM)
        _, err = p.communicate(timeout=60)
    assert "WARNING: ThreadSanitizer" not in err, err[-4000:]
    assert codes and set(codes) == {503}, set(codes)


@pytest.mark.slow
@pytest.mark.parametrize("target,binary,env", [
    ("asan", "bin/gpumon-exporter-asan", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                                          "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}),
    ("tsan", "bin/gpumon-exporter-tsan", {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}),
])
def test_sanitized_connection_flood_and_eviction(target, binary, env):
    """A connection flood at a 96-fd limit: the connection cap, evictions of idle connections in the
    middle of epoll batches, trickled headers timing out and scrapes getting in, under the
    sanitizers."""
    import resource

    from conftest import make_locked

    make_locked(target, jobs=8)
    port = _free_port()
    e = dict(os.environ, GPUMON_HTTP_HEADER_TIMEOUT_S="0.3", **env)
    p = subprocess.Popen([os.path.join(ROOT, binary), "--backend", "mock:gpus=2", "--interval", "0.02", "--listen",
                          f"127.0.0.1:{port}", "--http-threads", "2", "--log-level", "error"],
                         stderr=subprocess.PIPE, stdout=subprocess.DEVNULL, env=e, text=True,
                         preexec_fn=lambda: resource.setrlimit(resource.RLIMIT_NOFILE, (96, 96)))
    conns, got = [], 0
    try:
        deadline = time.time() + 30
        while time.time() < deadline:
            try:
                urllib.request.urlopen(f"http://127.0.0.1:{port}/healthz", timeout=1).read()
                break
            except OSError:
                time.sleep(0.1)
        for k in range(400):
            c = socket.socket()
            c.settimeout(2)
            try:
                c.connect(("127.0.0.1", port))
                if k % 3 == 0:
                    c.sendall(b"GET /metrics HTTP/1.1\r\n")  # a header that never ends
                conns.append(c)
            except OSError:
                c.close()
            if k % 50 == 0:
                try:
                    urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read()
                    got += 1
                except OSError:
                    pass
        time.sleep(1.0)
        assert p.poll() is None
    finally:
        for c in conns:
            c.close()
        p.send_signal(signal.SIGTERM)
        _, err = p.communicate(timeout=60)
    bad = _reports(err)
    assert not bad, err[-4000:]
    assert got >= 6, got


@pytest.mark.slow
@pytest.mark.parametrize("target,binary,env", [
    ("asan", "bin/gpumon-exporter-asan", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                                          "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}),
    ("tsan", "bin/gpumon-exporter-tsan", {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}),
])
def test_sanitized_https_serving(target, binary, env, tmp_path):
    """/metrics over HTTPS (csrc/core/tls.cpp TlsServer, the TLS branch of the HTTP loops) under
    ASan+UBSan and TSan: two loops serving concurrent verified scrapes and per-request filters over
    TLS, failed handshakes (plain HTTP and an untrusted scraper) mixed in, and the certificate files
    replaced every 0.15 s, so contexts are swapped while both loops create sessions. A bearer token
    guards /metrics too: its file is replaced as often (the same token, so every stamp change is a
    reload while both loops check requests), and requests with a wrong token are mixed in. No
    sanitizer report."""
    import ssl

    from conftest import make_locked
    from test_influx_tls import _ca, _leaf

    make_locked(target, jobs=8)
    d = str(tmp_path)
    _ca(d, "ca")
    _ca(d, "otherca")
    _leaf(d, "server", "ca", "DNS:localhost,IP:127.0.0.1")
    ctx = ssl.create_default_context(cafile=f"{d}/ca.pem")
    bad_ctx = ssl.create_default_context(cafile=f"{d}/otherca.pem")
    stop = threading.Event()
    port = _free_port()

    def intruders():  # handshake failures while the good scrapes run
        while not stop.is_set():
            for c in (None, bad_ctx):
                try:
                    if c is None:  # plain HTTP against the TLS port
                        s = socket.create_connection(("127.0.0.1", port), timeout=1)
                        s.sendall(b"GET /metrics HTTP/1.1\r\n\r\n")
                        s.recv(100)
                        s.close()
                    else:  # a scraper that does not trust the certificate
                        urllib.request.urlopen(f"https://localhost:{port}/metrics", timeout=1, context=c)
                except Exception:  # noqa: BLE001 -- refused by design
                    pass
                try:  # a trusted scraper with the wrong token (401)
                    urllib.request.urlopen(urllib.request.Request(f"https://localhost:{port}/metrics",
                                                                  headers={"Authorization": "Bearer nope"}),
                                           timeout=1, context=ctx)
                except Exception:  # noqa: BLE001 -- refused by design
                    pass
            time.sleep(0.02)

    import shutil

    os.makedirs(f"{d}/live")
    for src, dst in (("server.pem", "tls.crt"), ("server.key", "tls.key")):
        shutil.copy(f"{d}/{src}", f"{d}/live/{dst}")
    with open(f"{d}/token", "w") as f:
        f.write("sanitizer-token-0123456789\n")
    shutil.copy(f"{d}/token", f"{d}/live/token")

    def rotator():  # the kubelet's rename of the Secret's files, over and over: reloads while serving
        while not stop.is_set():
            for src, dst in (("server.pem", "tls.crt"), ("server.key", "tls.key"), ("token", "token")):
                shutil.copy(f"{d}/{src}", f"{d}/live/{dst}.new")
                os.replace(f"{d}/live/{dst}.new", f"{d}/live/{dst}")
            time.sleep(0.15)

    ts = [threading.Thread(target=intruders, daemon=True), threading.Thread(target=rotator, daemon=True)]
    for t in ts:
        t.start()
    try:
        rc, err = _run(os.path.join(ROOT, binary), dict(env, GPUMON_TLS_RELOAD_S="0.1"),
                       ("--tls-cert-file", f"{d}/live/tls.crt", "--tls-key-file", f"{d}/live/tls.key",
                        "--http-auth-token-file", f"{d}/live/token"), min_s=1.5,
                       ctx=ctx, port=port, token="sanitizer-token-0123456789")
    finally:
        stop.set()
        for t in ts:
            t.join(5)
    bad = _reports(err)
    assert not bad, err[-4000:]
    assert rc == 0, err[-2000:]


@pytest.mark.slow
@pytest.mark.parametrize("target,binary,env", [
    ("asan", "bin/gpumon-exporter-asan", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                                          "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}),
    ("tsan", "bin/gpumon-exporter-tsan", {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}),
])
def test_sanitized_https_push(target, binary, env, tmp_path):
    """The TLS push path (csrc/core/tls.cpp: the dlopen'd OpenSSL table, handshake, keep-alive
    reuse, close_notify on stop) under ASan+UBSan and TSan: pushes to a verifying TLS sink every
    20 ms with scrapes running, then a second run against a sink whose certificate does not verify
    (the failure / requeue / backoff path). No sanitizer report, every push of the good run
    delivered. LeakSanitizer sees OpenSSL's process-wide state too: the table is never unloaded."""
    from conftest import make_locked
    from test_influx_tls import _TlsSink, _ca, _leaf

    make_locked(target, jobs=8)
    d = str(tmp_path)
    _ca(d, "ca")
    _ca(d, "otherca")
    _leaf(d, "server", "ca", "DNS:localhost,IP:127.0.0.1")
    exe = os.path.join(ROOT, binary)
    # OpenSSL's own allocations are reachable process state (never unloaded), not leaks of ours
    san_env = dict(env)
    for ca, want_ok in ((f"{d}/ca.pem", True), (f"{d}/otherca.pem", False)):
        with _TlsSink(f"{d}/server.pem", f"{d}/server.key") as srv:
            rc, err = _run(exe, dict(san_env, GPUMON_INFLUX_CA_FILE=ca, GPUMON_INFLUX_TIMEOUT_S="0.5"),
                           ("--influx-url", f"https://localhost:{srv.port}/write?db=k8s", "--interval", "0.02"),
                           min_s=2.0, until=(lambda: len(srv.posts) >= 20) if want_ok else None)
        bad = _reports(err)
        assert not bad, err[-4000:]
        assert rc == 0, err[-2000:]
        if want_ok:
            assert len(srv.posts) >= 20 and not srv.handshake_errors, (len(srv.posts), srv.handshake_errors[:3])
            assert len({p["peer"] for p in srv.posts}) <= 2  # keep-alive: one connection (a reconnect at most)
        else:
            assert not srv.posts and srv.handshake_errors


@pytest.mark.slow
@pytest.mark.parametrize("target,binary,env", [
    ("asan", "bin/gpumon-exporter-asan", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                                          "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}),
    ("tsan", "bin/gpumon-exporter-tsan", {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}),
])
def test_sanitized_introspection_views(target, binary, env):
    """The loopback introspection server (csrc/core/exporter_debug.cpp) read continuously -- tick
    log, samples, rows, every GPU context, scrape durations, /debug/wait -- while the sampler ticks
    every 10 ms and /metrics is scraped: the views copy published state only (no report), and a
    /debug/wait in flight at SIGTERM does not hold the exit."""
    import http.client
    import json

    from conftest import make_locked

    make_locked(target, jobs=8)
    dport = _free_port()
    stop = threading.Event()
    got, errors = {}, []

    def reader():
        deadline = time.time() + 30
        while not stop.is_set():
            try:
                c = http.client.HTTPConnection("127.0.0.1", dport, timeout=10)
                for path in ("/debug/state", "/debug/ticks?since=0", "/debug/samples", "/debug/rows",
                             "/debug/procs", "/debug/scrapes?since=0", "/debug/wait?seq=0&timeout_s=0.05"):
                    c.request("GET", path)
                    r = c.getresponse()
                    body = r.read()
                    if r.status != 200:
                        errors.append((path, r.status))
                    got[path] = got.get(path, 0) + 1
                    json.loads(body)
                c.close()
            except (OSError, http.client.HTTPException):
                if time.time() > deadline and not got:
                    errors.append("debug server never answered")
                    return
                time.sleep(0.05)
            except ValueError as e:
                errors.append(("bad JSON", str(e)))

    t = threading.Thread(target=reader, daemon=True)
    t.start()
    try:
        rc, err = _run(os.path.join(ROOT, binary), dict(env),
                       ("--debug-listen", f"127.0.0.1:{dport}", "--interval", "0.01"), min_s=2.0,
                       until=lambda: min(got.values(), default=0) >= 20)
    finally:
        stop.set()
        t.join(15)
    assert not _reports(err), err[-4000:]
    assert rc == 0, err[-2000:]
    assert not errors, errors[:5]
    assert len(got) == 7 and min(got.values()) >= 5, got


@pytest.mark.slow
@pytest.mark.parametrize("target,binary,env", [
    ("asan", "bin/gpumon-exporter-asan", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                                          "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}),
    ("tsan", "bin/gpumon-exporter-tsan", {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}),
])
def test_sanitized_sysfs_fast_path_with_churning_kfd_queues(target, binary, env, tmp_path):
    """The real amdsmi backend over the fake libamd_smi with the sysfs fast path on a fake tree:
    gpu_metrics decode, the PCIe / activity accumulators, the KFD process scan with per-pid queue
    lists -- while another thread creates and removes KFD processes and their queue directories
    (readdir / open races of a live node) and /metrics is scraped. No report; the exporter keeps
    ticking and exits cleanly."""
    import shutil

    from conftest import make_locked
    from test_sysfs_fast import FAKE, _kfd_proc, _queues, make_tree

    make_locked(target, "fakes", jobs=8)
    sysr, procr = make_tree(tmp_path, gpus=2, procs=((4242, 0),))
    kfd = sysr / "class" / "kfd" / "kfd" / "proc"
    _queues(kfd / "4242", [36622, 36622])
    stop = threading.Event()
    churned = [0]

    def churn():
        i = 0
        while not stop.is_set():
            pid = 5000 + i % 7
            kp = kfd / str(pid)
            if kp.exists():
                shutil.rmtree(kp, ignore_errors=True)
            else:
                try:
                    _kfd_proc(sysr, pid, d=i % 2, occ=i % 50)
                    _queues(kp, [36622 + (i % 2)] * (i % 3))
                except OSError:
                    pass
            i += 1
            churned[0] = i
            time.sleep(0.003)

    t = threading.Thread(target=churn, daemon=True)
    t.start()
    try:
        e = dict(env, GPUMON_AMDSMI_LIB=FAKE, GPUMON_SYSFS_ROOT=str(sysr), GPUMON_PROCFS_ROOT=str(procr),
                 GPUMON_VERIFY_KFD="false", GPUMON_INIT_RETRY_S="0")
        for k in ("FAKE_AMDSMI_GPUS", "FAKE_AMDSMI_CPX", "FAKE_AMDSMI_NO_METRICS"):
            os.environ.pop(k, None)
        rc, err = _run(os.path.join(ROOT, binary), e, ("--backend", "amdsmi", "--interval", "0.01"), min_s=3.0)
    finally:
        stop.set()
        t.join(10)
    assert not _reports(err), err[-4000:]
    assert rc == 0, err[-2000:]
    assert churned[0] > 100
