"""Plain-Docker nodes: the native Docker Engine listing (csrc/core/docker_lite.cpp) against a fake
daemon on a unix socket, its JSON / HTTP/1.x readers against Python's own, and the exporter's
poller feeding pod_gpu rows. The reference read the same container labels through `docker inspect`
(/root/reference/gpu.py:86-88,184-195): io.kubernetes.pod.{name,namespace} for the podname /
namespace tags and the `mlgpu` opt-in label (gpu.py:185-189)."""

import json
import os
import socketserver
import threading
from http.server import BaseHTTPRequestHandler

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from gpumon.export import promtext

CID_K8S = "1a" * 32
CID_PLAIN = "2b" * 32
CID_OTHER = "3c" * 32


def _container(cid, name, labels, **extra):
    c = {"Id": cid, "Names": ["/" + name], "Image": "rocm/pytorch:latest", "ImageID": "sha256:" + "0" * 64,
         "Command": "python train.py", "Created": 1700000000, "Ports": [{"PrivatePort": 8888, "Type": "tcp"}],
         "Labels": labels, "State": "running", "Status": "Up 3 hours",
         "HostConfig": {"NetworkMode": "default", "Annotations": None},
         "NetworkSettings": {"Networks": {"bridge": {"IPAddress": "172.17.0.2", "MacAddress": "02:42:ac:11:00:02",
                                                     "IPPrefixLen": 16, "Aliases": None}}},
         "Mounts": [{"Type": "bind", "Source": "/dev/kfd", "Destination": "/dev/kfd", "RW": True}]}
    c.update(extra)
    return c


K8S_LABELS = {"io.kubernetes.pod.name": "turing-gpu-notebook-alice-1-2", "io.kubernetes.pod.namespace": "ml",
              "io.kubernetes.container.name": "nb", "io.kubernetes.pod.uid": "uid-a", "mlgpu": "mlgpu"}


def test_parse_realistic_listing(core):
    body = json.dumps([_container(CID_K8S, "k8s_nb_turing-gpu-notebook-alice-1-2_ml_uid-a_0", K8S_LABELS),
                       _container(CID_PLAIN, "bench", {"mlgpu": "mlgpu", "owner": "böb \U0001F600"}),
                       _container(CID_OTHER, "nolabels", None, Names=None)]).encode()
    cs = core.docker_parse_containers(body)
    assert [c["id"] for c in cs] == [CID_K8S, CID_PLAIN, CID_OTHER]
    assert cs[0]["name"] == "k8s_nb_turing-gpu-notebook-alice-1-2_ml_uid-a_0" and cs[0]["labels"] == K8S_LABELS
    assert cs[1]["labels"]["owner"] == "böb \U0001F600" and cs[1]["state"] == "running"
    assert cs[2]["name"] == "" and cs[2]["labels"] == {}
    assert core.docker_parse_containers(b" [ ] ") == []


@pytest.mark.parametrize("bad", [b"", b"{}", b"[", b"[{]", b'[{"Id": "x"', b'[{"Id": "x"}] trailing',
                                 b'[{"Id": "\\ud800"}]', b'[{"Id": "\\q"}]', b'[{"Id": "a\x01"}]',
                                 b'[{"Labels": {"a": }}]', b'[{"X": 1.}]', b'[{"X": -}]', b'[{"X": tru}]',
                                 b"[" + b"[" * 100 + b"]" * 100 + b"]"])
def test_malformed_listing_is_an_error(core, bad):
    with pytest.raises(ValueError):
        core.docker_parse_containers(bad)


_text = st.text(st.characters(blacklist_categories=("Cs",)), max_size=12)


@settings(max_examples=200, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(st.lists(st.fixed_dictionaries(
    {"Id": st.text("0123456789abcdef", min_size=1, max_size=64), "Names": st.lists(_text, max_size=3),
     "Labels": st.one_of(st.none(), st.dictionaries(_text, _text, max_size=4)),
     "Junk": st.recursive(st.one_of(st.none(), st.booleans(), st.integers(), st.floats(allow_nan=False,
                                                                                         allow_infinity=False), _text),
                          lambda c: st.one_of(st.lists(c, max_size=3), st.dictionaries(_text, c, max_size=3)),
                          max_leaves=8)}), max_size=4), st.booleans())
def test_parser_agrees_with_python_json(core, containers, ascii_only):
    got = core.docker_parse_containers(json.dumps(containers, ensure_ascii=ascii_only).encode())
    assert [c["id"] for c in got] == [c["Id"] for c in containers]
    for g, c in zip(got, containers):
        assert g["labels"] == (c["Labels"] or {})
        first = c["Names"][0] if c["Names"] else ""
        assert g["name"] == (first[1:] if len(first) > 1 and first[0] == "/" else first)


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(st.binary(max_size=200))
def test_parser_never_crashes_on_garbage(core, data):
    try:
        core.docker_parse_containers(data)
    except ValueError:
        pass


def test_http1_response_framing(core):
    body = b'[{"Id": "ab"}]'
    cl = b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n%sEXTRA" % (len(body), body)
    assert core.http1_parse_response(cl) == (200, body)
    ch = b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n5\r\n[{\"Id\r\n9\r\n\": \"ab\"}]\r\n0\r\n\r\n"
    assert core.http1_parse_response(ch) == (200, body)
    assert core.http1_parse_response(b"HTTP/1.0 404 Not Found\r\n\r\nnope") == (404, b"nope")
    assert core.http1_parse_response(cl, eof=False) == (200, body)  # framed: complete before EOF
    with pytest.raises(ValueError, match="incomplete"):  # close-delimited: only complete at EOF
        core.http1_parse_response(b"HTTP/1.0 200 OK\r\n\r\n[]", eof=False)
    for bad in (b"HTTP/1.1 200 OK\r\n", b"garbage\r\n\r\n", b"HTTP/1.1 200 OK\r\nContent-Length: 99\r\n\r\nshort",
                b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n"):
        with pytest.raises(ValueError):
            core.http1_parse_response(bad)


@pytest.mark.parametrize("raw,error", [
    (b"HTTP/1.1 200 OK\r\nContent-Length: x\r\n\r\n", "bad Content-Length"),
    (b"HTTP/1.1 200 OK\r\nContent-Length: -4\r\n\r\nabcd", "bad Content-Length"),
    (b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nab", "truncated chunk"),
    (b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n5", "truncated chunk size"),
    (b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\nfffffffff\r\n", "bad chunk size"),
    (b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n", "bad chunk size"),
    (b"HTTP/1.1 200 OK\r\nContent-Length: 99\r\n\r\nshort", "truncated"),
    (b"HTTP/2 200\r\n\r\n", "bad HTTP status line"),
])
def test_http1_response_errors_are_named(core, raw, error):
    with pytest.raises(ValueError, match=error):
        core.http1_parse_response(raw)


@settings(max_examples=300, deadline=None)
@given(st.binary(max_size=200), st.booleans())
def test_http1_reader_never_crashes_on_garbage(data, eof):
    from gpumon import core as _core

    for raw in (data, b"HTTP/1.1 200 OK\r\n" + data, b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n" + data):
        try:
            status, body = _core().http1_parse_response(raw, eof=eof)
            assert isinstance(body, bytes) and len(body) <= len(raw)
        except ValueError:
            pass


class _RawDaemon:
    """A unix-socket peer that reads the request, then plays `script` (bytes, "close", or a float
    to sleep) and holds the connection: the daemon misbehaviours a framed reader must survive."""

    def __init__(self, path, script):
        import socket as so

        if os.path.exists(path):
            os.unlink(path)
        self.path, self.script, self.stop = path, script, threading.Event()
        self.srv = so.socket(so.AF_UNIX, so.SOCK_STREAM)
        self.srv.bind(path)
        self.srv.listen(2)
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _run(self):
        import time

        conn, _ = self.srv.accept()
        try:
            req = b""
            while b"\r\n\r\n" not in req:
                req += conn.recv(4096)
            for step in self.script:
                if step == "close":
                    return
                if isinstance(step, float):
                    time.sleep(step)
                else:
                    conn.sendall(step)
            self.stop.wait(10)
        except OSError:
            pass
        finally:
            conn.close()

    def close(self):
        self.stop.set()
        self.srv.close()
        self.t.join(5)
        os.unlink(self.path)


@pytest.mark.parametrize("script,error", [
    ([b"HTTP/1.1 200 OK\r\nContent-Length: 10\r\n\r\n[]"], "read timed out"),  # short and silent
    ([b"HTTP/1.1 200 OK\r\n"], "read timed out"),  # headers never end
    (["close"], "truncated HTTP response header"),  # hangs up before answering
    ([b"HTTP/1.1 200 OK\r\nContent-Length: 5\r\n\r\n[", "close"], "truncated"),
    ([b"HTTP/1.0 200 OK\r\n\r\n" + b" " * (1 << 20)] * 65, "response too large"),  # never ends
])
def test_native_docker_reader_bounds_a_misbehaving_daemon(core, script, error):
    import time

    d = _RawDaemon(_sock("raw"), script)
    # the endless daemon must be cut off by the size bound (64 MiB), not by the clock: give its read
    # time enough for 64 MiB on a loaded host
    timeout_ms = 3000 if error == "response too large" else 400
    try:
        t0 = time.monotonic()
        with pytest.raises(RuntimeError, match=error):
            core.docker_list(d.path, timeout_ms=timeout_ms)
        assert time.monotonic() - t0 < timeout_ms / 1000 + 2.6
    finally:
        d.close()


class FakeDocker:
    """Docker Engine API subset on a unix socket: GET /containers/json (others 404). `containers`
    is a listing, or a callable returning the raw body of each response."""

    def __init__(self, path, containers, status=200, chunked=False, keep_open=False, inspect=None):
        self.path, self.containers, self.status, self.chunked, self.requests = path, containers, status, chunked, []
        self.inspect = inspect or {}  # container id -> GET /containers/{id}/json object
        outer = self

        class H(BaseHTTPRequestHandler):
            # keep_open: an HTTP/1.1 handler that keeps the connection after answering, even to 1.0
            protocol_version = "HTTP/1.1" if keep_open else "HTTP/1.0"

            def do_GET(self):  # noqa: N802
                outer.requests.append((self.command, self.path, self.request_version))
                parts = self.path.split("/")
                if len(parts) == 4 and parts[1] == "containers" and parts[3] == "json" and parts[2] in outer.inspect:
                    body = json.dumps(outer.inspect[parts[2]]).encode()
                    self.send_response(200)
                    self.send_header("Content-Type", "application/json")
                    self.send_header("Content-Length", str(len(body)))
                    self.end_headers()
                    self.wfile.write(body)
                    return
                if self.path != "/containers/json":
                    self.send_error(404)
                    return
                if outer.status != 200:
                    body = b'{"message":"denied"}'
                elif callable(outer.containers):  # raw bodies (mutation fuzzing of the native reader)
                    body = outer.containers()
                else:
                    body = json.dumps(outer.containers).encode()
                self.send_response(outer.status)
                self.send_header("Content-Type", "application/json")
                if outer.chunked:  # a daemon that chunks regardless of the request version
                    self.send_header("Transfer-Encoding", "chunked")
                    self.end_headers()
                    for i in range(0, len(body), 7):
                        part = body[i:i + 7]
                        self.wfile.write(b"%x\r\n%s\r\n" % (len(part), part))
                    self.wfile.write(b"0\r\n\r\n")
                else:
                    self.send_header("Content-Length", str(len(body)))
                    self.end_headers()
                    self.wfile.write(body)

            def address_string(self):
                return "unix"

            def log_message(self, *a):
                pass

        class S(socketserver.ThreadingMixIn, socketserver.UnixStreamServer):
            daemon_threads = True

        if os.path.exists(path):  # left behind by a killed run
            os.unlink(path)
        self.srv = S(path, H)
        self.t = threading.Thread(target=self.srv.serve_forever, daemon=True)

    def __enter__(self):
        self.t.start()
        return self

    def __exit__(self, *a):
        self.srv.shutdown()
        self.srv.server_close()
        os.unlink(self.path)


def _sock(tag):
    return f"/tmp/gpumon-docker-{tag}-{os.getpid()}.sock"


@pytest.mark.parametrize("chunked,keep_open", [(False, False), (True, False), (False, True), (True, True)])
def test_native_docker_list(core, chunked, keep_open):
    import time

    cs = [_container(CID_K8S, "k8s_nb", K8S_LABELS), _container(CID_PLAIN, "bench", {"mlgpu": "mlgpu"})]
    with FakeDocker(_sock(f"l{int(chunked)}{int(keep_open)}"), cs, chunked=chunked, keep_open=keep_open) as d:
        t0 = time.monotonic()
        got = core.docker_list(d.path, timeout_ms=3000)
        assert time.monotonic() - t0 < 1.0  # a framed response ends the read, not the timeout
    assert [(c["id"], c["name"]) for c in got] == [(CID_K8S, "k8s_nb"), (CID_PLAIN, "bench")]
    assert d.requests == [("GET", "/containers/json", "HTTP/1.0")]  # the one read-only request


def test_native_docker_list_errors(core):
    with FakeDocker(_sock("e"), [], status=403) as d:
        with pytest.raises(RuntimeError, match="HTTP 403"):
            core.docker_list(d.path)
    with pytest.raises(RuntimeError, match="connect"):
        core.docker_list("/tmp/gpumon-no-such-docker.sock")


def _fake_proc(root, pid, cgroup_line):
    d = root / str(pid)
    d.mkdir(parents=True)
    (d / "stat").write_text(f"{pid} (python) S 1 1 1 0 -1 0 0 0 0 0 0 0 0 0 20 0 1 0 777 0 0\n")
    (d / "cgroup").write_text(cgroup_line + "\n")


def test_exporter_attributes_docker_containers(core, tmp_path):
    """Docker-only node: a dockershim-era k8s container (io.kubernetes.* labels, cgroup v1 docker
    path) and a plain `docker run` container (cgroup v2 systemd scope) are both attributed from the
    Docker listing; the `mlgpu` opt-in gate sees the container labels as in gpu.py:185-189."""
    _fake_proc(tmp_path, 1000, f"12:devices:/kubepods/burstable/poduid-a/{CID_K8S}")
    _fake_proc(tmp_path, 2000, f"0::/system.slice/docker-{CID_PLAIN}.scope")
    _fake_proc(tmp_path, 3000, f"0::/system.slice/docker-{CID_OTHER}.scope")
    cs = [_container(CID_K8S, "k8s_nb", K8S_LABELS),
          _container(CID_PLAIN, "bench", {"mlgpu": "mlgpu", "team": "q"}),
          _container(CID_OTHER, "noopt", {})]
    with FakeDocker(_sock("x"), cs) as d:
        ex = core.Exporter({"backend": "mock:gpus=2", "serve_http": False, "interval_s": 0, "host": "n1",
                            "procfs_root": str(tmp_path), "docker_socket": "unix://" + d.path,
                            "opt_in": "mlgpu=mlgpu", "label_allowlist": ["team"]})
        ex.start()
        try:
            ex.mock_set_procs([{"pid": 1000, "device": 0, "name": "python", "vram_bytes": 5 << 30},
                               {"pid": 2000, "device": 1, "name": "bench", "vram_bytes": 1 << 30},
                               {"pid": 3000, "device": 1, "name": "other", "vram_bytes": 1 << 30}])
            ex.tick()
            rows = {r["pid"]: r for r in ex.pod_rows() if not r["idle"]}
            assert set(rows) == {"1000", "2000"}  # the container without mlgpu=mlgpu is gated out
            k = rows["1000"]
            assert (k["podname"], k["namespace"], k["container"], k["user_name"], k["containerid"]) == \
                ("turing-gpu-notebook-alice-1-2", "ml", "nb", "alice", CID_K8S[:12])
            p = rows["2000"]
            assert (p["podname"], p["namespace"], p["container"], p["containerid"]) == ("-", "-", "bench", CID_PLAIN[:12])
            fam = promtext.parse(ex.metrics_text())
            assert promtext.one(fam, "gpumon_docker_up") == 1 and promtext.one(fam, "gpumon_docker_containers") == 3
            assert promtext.one(fam, "gpumon_docker_http_status") == 200
        finally:
            ex.stop()
    assert d.requests and all(r[0] == "GET" and r[2] == "HTTP/1.0" for r in d.requests)
    assert {r[1] for r in d.requests} <= {"/containers/json"} | {f"/containers/{c}/json" for c in (CID_K8S, CID_PLAIN, CID_OTHER)}


def test_exporter_reports_a_failing_docker_daemon(core, tmp_path):
    with FakeDocker(_sock("f"), [], status=500) as d:
        ex = core.Exporter({"backend": "mock:gpus=1", "serve_http": False, "interval_s": 0,
                            "procfs_root": str(tmp_path), "docker_socket": d.path})
        ex.start()
        try:
            ex.tick()
            fam = promtext.parse(ex.metrics_text())
            assert promtext.one(fam, "gpumon_docker_up") == 0 and promtext.one(fam, "gpumon_docker_http_status") == 500
        finally:
            ex.stop()


def test_docker_socket_is_never_autodetected():
    """Opt-in only, in both planes: the socket is root-equivalent (the reference mounted it,
    gpu_monitor.yaml:24-28,38-44); --docker / docker_socket turn it on."""
    import subprocess

    from gpumon.config import Config

    assert Config().docker_socket == ""
    binary = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bin/gpumon-exporter")
    r = subprocess.run([binary, "--print-config"], capture_output=True, text=True, timeout=30, check=True)
    assert json.loads(r.stdout)["docker_socket"] == ""
    r = subprocess.run([binary, "--docker", "/run/docker.sock", "--print-config"], capture_output=True, text=True,
                       timeout=30, check=True)
    assert json.loads(r.stdout)["docker_socket"] == "/run/docker.sock"


def _inspect(cid, devices=(), env=()):
    return {"Id": cid, "Created": "2026-10-17T00:00:00Z", "Path": "python", "Args": ["train.py"],
            "State": {"Status": "running", "Pid": 4242},
            "Config": {"Hostname": "x", "Env": list(env) + ["PATH=/usr/bin"], "Labels": {"a": "b"},
                       "Cmd": ["python"], "Volumes": None},
            "HostConfig": {"Binds": None, "Privileged": False,
                           "Devices": [{"PathOnHost": p, "PathInContainer": p, "CgroupPermissions": "rwm"}
                                       for p in devices],
                           "DeviceRequests": None, "Ulimits": [{"Name": "memlock", "Soft": -1, "Hard": -1}]},
            "Mounts": [], "NetworkSettings": {"Ports": {}}}


def test_parse_inspect(core):
    d = core.docker_parse_inspect(json.dumps(_inspect(CID_PLAIN, ["/dev/kfd", "/dev/dri/renderD129"],
                                                      ["AMD_VISIBLE_DEVICES=1"])).encode())
    assert d["id"] == CID_PLAIN and d["devices"] == ["/dev/kfd", "/dev/dri/renderD129"]
    assert "AMD_VISIBLE_DEVICES=1" in d["env"]
    d = core.docker_parse_inspect(b'{"Id": "ab", "Config": null, "HostConfig": {"Devices": null}}')
    assert d["devices"] == [] and d["env"] == []
    for bad in (b"[]", b'{"HostConfig": {"Devices": [{"PathOnHost": 1}]', b'{"Config": {"Env": [1,}}'):
        with pytest.raises(ValueError):
            core.docker_parse_inspect(bad)


def test_container_gpus_mapping(core):
    st = [{"index": i, "drm_card": i, "drm_render": 128 + i, "bdf": f"0000:{0x05 + 0x20 * i:02x}:00.0",
           "uuid": f"uuid-{i}"} for i in range(4)]
    g = core.docker_container_gpus
    assert g(["/dev/kfd", "/dev/dri/renderD130"], [], st) == [2]
    assert g(["/dev/dri/card1", "/dev/dri/renderD129"], [], st) == [1]
    assert g(["/dev/dri/"], [], st) == [0, 1, 2, 3]  # the whole directory
    assert g(["/dev/kfd"], [], st) == []  # KFD alone names no GPU
    assert g([], ["AMD_VISIBLE_DEVICES=all"], st) == [0, 1, 2, 3]
    assert g([], ["AMD_VISIBLE_DEVICES=3,0,9"], st) == [0, 3]  # 9: no such GPU
    assert g([], ["AMD_VISIBLE_DEVICES=uuid-2,0000:25:00.0"], st) == [1, 2]
    assert g(["/dev/dri/renderD999", "/dev/dri/renderDx"], ["OTHER=1"], st) == []


def test_exporter_idle_rows_for_docker_gpu_containers(core, tmp_path):
    """The reference found allocated-but-idle GPUs by running `nvidia-smi -L` inside every opted-in
    container (gpu.py:220-253, docker exec). On a Docker node the exporter reads which GPUs each
    container was given (device mappings or AMD_VISIBLE_DEVICES, one inspect per new container) and
    emits the idle rows for those without a GPU process."""
    _fake_proc(tmp_path, 2000, f"0::/system.slice/docker-{CID_PLAIN}.scope")
    cs = [_container(CID_PLAIN, "busy", {"mlgpu": "mlgpu"}),
          _container(CID_OTHER, "waiting", {"mlgpu": "mlgpu"}),
          _container(CID_K8S, "k8s_nb", K8S_LABELS)]
    insp = {CID_PLAIN: _inspect(CID_PLAIN, ["/dev/kfd", "/dev/dri/renderD128"]),
            CID_OTHER: _inspect(CID_OTHER, ["/dev/kfd"], ["AMD_VISIBLE_DEVICES=1"]),
            CID_K8S: _inspect(CID_K8S, [])}
    with FakeDocker(_sock("a"), cs, inspect=insp) as d:
        ex = core.Exporter({"backend": "mock:gpus=2", "serve_http": False, "interval_s": 0, "host": "n1",
                            "procfs_root": str(tmp_path), "docker_socket": d.path, "opt_in": "mlgpu=mlgpu"})
        ex.start()
        try:
            ex.mock_set_procs([{"pid": 2000, "device": 0, "name": "bench", "vram_bytes": 1 << 30}])
            ex.tick()
            rows = sorted((r["dev"], r["idle"], r["container"], r["containerid"]) for r in ex.pod_rows())
            assert rows == [(0, False, "busy", CID_PLAIN[:12]), (1, True, "waiting", CID_OTHER[:12])], rows
            fam = promtext.parse(ex.metrics_text())
            assert promtext.one(fam, "gpumon_gpus", state="allocated") == 2
            assert promtext.one(fam, "gpumon_gpus", state="allocated_idle") == 1
            assert promtext.one(fam, "gpumon_docker_inspect_errors") == 0
        finally:
            ex.stop()
    inspects = [r[1] for r in d.requests if r[1] != "/containers/json"]
    assert sorted(inspects) == sorted(f"/containers/{c}/json" for c in insp)  # once per container


def test_native_docker_reader_on_a_full_listener_backlog(core):
    """A daemon that stopped accepting: once its listen backlog is full, a non-blocking unix
    connect fails with EAGAIN (no connection was made); the reader says so at once."""
    import socket as so
    import time

    path = _sock("backlog")
    if os.path.exists(path):
        os.unlink(path)
    srv = so.socket(so.AF_UNIX, so.SOCK_STREAM)
    srv.bind(path)
    srv.listen(0)
    fillers = []
    try:
        for _ in range(8):  # fill the backlog (never accepted)
            c = so.socket(so.AF_UNIX, so.SOCK_STREAM)
            c.setblocking(False)
            try:
                c.connect(path)
            except (BlockingIOError, OSError):
                c.close()
                break
            fillers.append(c)
        t0 = time.monotonic()
        with pytest.raises(RuntimeError, match="listener backlog full"):
            core.docker_list(path, timeout_ms=3000)
        assert time.monotonic() - t0 < 1.0
    finally:
        for c in fillers:
            c.close()
        srv.close()
        os.unlink(path)
