#!/usr/bin/env python3
"""HTTPS push soak of the image's entrypoint: `bin/gpumon-exporter` at 10 Hz pushes every tick to a
local InfluxDB stand-in over verified TLS, while a gzip scraper reads /metrics. The stand-in is a
Python `ssl` server with a CA made by the `openssl` CLI.

The sink misbehaves on a schedule, the way a real endpoint behind a load balancer does:
- every 50th answer carries `Connection: close`, so the exporter must reconnect and handshake again;
- every 200th request gets a 503, which must be retried in order.

Every 30 s one JSON line goes to stdout with the exporter's RSS, fds and threads, the
push counters it exports, the sink's counts and the scrape p99. The final summary is the last line.
A leak across reconnects shows up as a trend in fds or RSS. A lost or reordered batch shows up as a
gap in the sink's tick sequence.

With `--serve-tls` the exporter also serves /metrics over HTTPS, and the scraper verifies it. With
`--rotate-every S` the serving certificate is re-issued and swapped into place every S seconds, the
way the kubelet updates a mounted Secret, while scrapes run. With `--token` /metrics also needs a
bearer token; on each rotation the token is replaced with an overlap (old and new line, the
scraper moves to the new one, the old line goes), which must refuse no scrape.

On a GPU box: `--backend amdsmi` (default) next to the mixed K2 load. On CPU: `--backend mock`.
"""

import argparse
import http.client
import http.server
import json
import os
import shutil
import socket
import ssl
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _openssl(*args, cwd):
    subprocess.run(["openssl", *args], cwd=cwd, check=True, capture_output=True, timeout=60)


def make_pki(d):
    _openssl("req", "-x509", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes", "-days", "2",
             "-keyout", "ca.key", "-out", "ca.pem", "-subj", "/CN=soak-ca", cwd=d)
    _openssl("req", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes", "-keyout", "server.key",
             "-out", "server.csr", "-subj", "/CN=localhost", cwd=d)
    with open(os.path.join(d, "server.ext"), "w") as fh:
        fh.write("basicConstraints=CA:FALSE\nsubjectAltName=DNS:localhost,IP:127.0.0.1\nextendedKeyUsage=serverAuth\n")
    _openssl("x509", "-req", "-in", "server.csr", "-CA", "ca.pem", "-CAkey", "ca.key", "-CAcreateserial", "-days", "2",
             "-out", "server.pem", "-extfile", "server.ext", cwd=d)
    # a scraper's client certificate (mutual TLS, --mtls)
    _openssl("req", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes", "-keyout", "client.key",
             "-out", "client.csr", "-subj", "/CN=prometheus", cwd=d)
    with open(os.path.join(d, "client.ext"), "w") as fh:
        fh.write("basicConstraints=CA:FALSE\nextendedKeyUsage=clientAuth\n")
    _openssl("x509", "-req", "-in", "client.csr", "-CA", "ca.pem", "-CAkey", "ca.key", "-CAcreateserial", "-days", "2",
             "-out", "client.pem", "-extfile", "client.ext", cwd=d)
    return {k: os.path.join(d, f"{k}.pem") for k in ("ca", "server", "client")} | {
        "server_key": os.path.join(d, "server.key"), "client_key": os.path.join(d, "client.key")}


class Sink(http.server.ThreadingHTTPServer):
    daemon_threads = True

    def __init__(self, pki, close_every, fail_every):
        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def do_POST(self):  # noqa: N802
                srv = self.server
                n = int(self.headers.get("Content-Length", 0))
                body = self.rfile.read(n).decode()
                with srv.lock:
                    srv.requests += 1
                    k = srv.requests
                    fail = srv.fail_every and k % srv.fail_every == 0
                    if not fail:
                        srv.posts += 1
                        srv.lines += body.count("\n")
                        srv.node_lines += sum(1 for l in body.splitlines() if l.startswith("node_gpu,"))
                        # one batch per tick, in order: the node_gpu timestamps never go backwards
                        ts = [int(l.rsplit(" ", 1)[1]) for l in body.splitlines() if l.startswith("node_gpu,")]
                        if ts and srv.last_ts and min(ts) < srv.last_ts:
                            srv.reordered += 1
                        if ts:
                            srv.last_ts = max(ts)
                self.send_response(503 if fail else 204)
                self.send_header("Content-Length", "0")
                if srv.close_every and k % srv.close_every == 0:
                    self.send_header("Connection", "close")
                    self.close_connection = True
                self.end_headers()

            def log_message(self, *a):
                pass

        super().__init__(("127.0.0.1", 0), H)
        self.lock = threading.Lock()
        self.requests = self.posts = self.lines = self.node_lines = self.reordered = self.handshakes = 0
        self.last_ts = 0
        self.close_every, self.fail_every = close_every, fail_every
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(pki["server"], pki["server_key"])
        self.ctx = ctx
        self.port = self.server_address[1]
        threading.Thread(target=self.serve_forever, daemon=True).start()

    def get_request(self):
        sock, addr = self.socket.accept()
        return self.ctx.wrap_socket(sock, server_side=True, do_handshake_on_connect=False), addr

    def process_request_thread(self, request, client_address):
        try:
            request.do_handshake()
            with self.lock:
                self.handshakes += 1
        except (ssl.SSLError, OSError):
            self.shutdown_request(request)
            return
        super().process_request_thread(request, client_address)


def proc_stats(pid):
    rss = 0
    with open(f"/proc/{pid}/status") as f:
        for l in f:
            if l.startswith("VmRSS:"):
                rss = int(l.split()[1]) * 1024
    return {"rss_mb": round(rss / 2 ** 20, 2), "fds": len(os.listdir(f"/proc/{pid}/fd")),
            "threads": len(os.listdir(f"/proc/{pid}/task"))}


def _auth(token):
    return {"Authorization": f"Bearer {token['value']}"} if token and token.get("value") else {}


def push_counters(port, ctx=None, token=None):
    from gpumon.export import promtext

    c = (http.client.HTTPSConnection("localhost", port, context=ctx, timeout=5) if ctx
         else http.client.HTTPConnection("127.0.0.1", port, timeout=5))
    c.request("GET", "/metrics?include=gpumon_influx_*,gpumon_ticks_total,gpumon_http_tls_*,gpumon_http_auth_*",
              headers=_auth(token))
    fam = promtext.parse(c.getresponse().read().decode())
    c.close()
    out = {"ticks": promtext.one(fam, "gpumon_ticks_total"), "influx_up": promtext.one(fam, "gpumon_influx_up")}
    for _, labels, v in fam.get("gpumon_influx_push_total", {}).get("samples", []):
        out["push_" + labels.get("result", "?")] = v
    if ctx:
        out["tls_handshake_failures"] = promtext.one(fam, "gpumon_http_tls_handshake_failures_total")
        for _, labels, v in fam.get("gpumon_http_tls_reloads_total", {}).get("samples", []):
            out["tls_reloads_" + labels.get("result", "?")] = v
    if token:
        out["auth_failures"] = sum(v for _, _, v in fam.get("gpumon_http_auth_failures_total", {}).get("samples", []))
        for _, labels, v in fam.get("gpumon_http_auth_token_reloads_total", {}).get("samples", []):
            out["auth_reloads_" + labels.get("result", "?")] = v
    return out


def probe_without_cert(port, ctx_nocert):
    """What the kubelet's probes and a scraper without a client certificate get under mutual TLS:
    (health / readiness statuses, /metrics status)."""
    out = []
    for path in ("/healthz", "/readyz", "/metrics"):
        c = http.client.HTTPSConnection("localhost", port, context=ctx_nocert, timeout=5)
        try:
            c.request("GET", path)
            r = c.getresponse()
            r.read()
            out.append(r.status)
        except (OSError, ssl.SSLError, http.client.HTTPException):
            out.append(-1)
        finally:
            c.close()
    return out[:2], out[2]


def tls_scrapes(port, ctx, seconds, rate_hz, token=None):
    """Verified HTTPS scrapes with gzip over one keep-alive connection (reopened after an error),
    paced at rate_hz, with the bearer token current at each request: (latencies, errors)."""
    lat, errors, conn = [], 0, None
    period, t_next, end = 1.0 / rate_hz, time.monotonic(), time.monotonic() + seconds
    while time.monotonic() < end:
        time.sleep(max(0.0, t_next - time.monotonic()))
        t_next += period
        try:
            if conn is None:
                conn = http.client.HTTPSConnection("localhost", port, context=ctx, timeout=5)
            t = time.perf_counter()
            conn.request("GET", "/metrics", headers={"Accept-Encoding": "gzip", **_auth(token)})
            r = conn.getresponse()
            r.read()
            if r.status != 200:
                raise OSError(f"HTTP {r.status}")
            lat.append(time.perf_counter() - t)
        except (OSError, ssl.SSLError, http.client.HTTPException):
            errors += 1
            if conn is not None:
                conn.close()
            conn = None
    if conn is not None:
        conn.close()
    return lat, errors


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=10.0)
    ap.add_argument("--interval", type=float, default=0.1)
    ap.add_argument("--backend", default="amdsmi")
    ap.add_argument("--window", type=float, default=30.0)
    ap.add_argument("--scrape-rate", type=float, default=20.0)
    ap.add_argument("--close-every", type=int, default=50)
    ap.add_argument("--fail-every", type=int, default=200)
    ap.add_argument("--serve-tls", action="store_true", help="serve /metrics over HTTPS and scrape it verified")
    ap.add_argument("--rotate-every", type=float, default=0.0,
                    help="with --serve-tls: re-issue and swap the serving certificate every S seconds (0 = never)")
    ap.add_argument("--mtls", action="store_true",
                    help="with --serve-tls: mutual TLS (tls_client_ca_file); the scraper presents a client "
                         "certificate, and each window the probes and a certificate-less /metrics are checked")
    ap.add_argument("--token", action="store_true",
                    help="with --serve-tls: /metrics needs a bearer token, rotated with an overlap at each rotation")
    a = ap.parse_args()
    if (a.token or a.mtls) and not a.serve_tls:
        raise SystemExit("push_soak: --token / --mtls need --serve-tls")
    if shutil.which("openssl") is None:
        raise SystemExit("push_soak: the openssl CLI is needed for the test CA")

    from gpumon import core as _core

    core = _core()
    tmp = tempfile.mkdtemp(prefix="gpumon-push-soak-")
    pki = make_pki(tmp)
    sink = Sink(pki, a.close_every, a.fail_every)
    load = None
    if a.backend.startswith("amdsmi"):
        from gpumon.ops.load import SyntheticLoad

        load = SyntheticLoad(0, "mixed").start()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, INFLUXDB_URL=f"https://localhost:{sink.port}/write?db=k8s", GPUMON_INFLUX_CA_FILE=pki["ca"],
               NODE_NAME="soak-node", GPUMON_TLS_RELOAD_S="1")
    args = [os.path.join(ROOT, "bin", "gpumon-exporter"), "--backend", a.backend, "--interval", str(a.interval),
            "--listen", f"127.0.0.1:{port}", "--log-level", "error"]
    ctx = None
    rotations = token_rotations = 0
    token = {"value": "soak-token-0000000000000000"} if a.token else None
    stop_rotation = threading.Event()
    if a.serve_tls:
        live = os.path.join(tmp, "live")
        os.makedirs(live)
        shutil.copy(pki["server"], os.path.join(live, "tls.crt"))
        shutil.copy(pki["server_key"], os.path.join(live, "tls.key"))
        args += ["--tls-cert-file", os.path.join(live, "tls.crt"), "--tls-key-file", os.path.join(live, "tls.key")]
        ctx = ssl.create_default_context(cafile=pki["ca"])
        ctx_nocert = None
        if a.mtls:
            args += ["--tls-client-ca-file", pki["ca"]]
            ctx_nocert = ssl.create_default_context(cafile=pki["ca"])
            ctx.load_cert_chain(pki["client"], pki["client_key"])
        tok_file = os.path.join(live, "token")

        def put_token(text):  # the kubelet's rename of the Secret's file
            with open(tok_file + ".new", "w") as f:
                f.write(text)
            os.replace(tok_file + ".new", tok_file)

        if token:
            put_token(token["value"] + "\n")
            args += ["--http-auth-token-file", tok_file]

        def rotate():  # a renewal: same key, new certificate, renamed into place
            nonlocal rotations, token_rotations
            while a.rotate_every > 0 and not stop_rotation.wait(a.rotate_every):
                _openssl("x509", "-req", "-in", "server.csr", "-CA", "ca.pem", "-CAkey", "ca.key", "-CAcreateserial",
                         "-days", "2", "-out", os.path.join(live, "tls.crt.new"), "-extfile", "server.ext", cwd=tmp)
                os.replace(os.path.join(live, "tls.crt.new"), os.path.join(live, "tls.crt"))
                rotations += 1
                if token:  # overlap: both tokens, the scraper moves, then only the new one
                    new = f"soak-token-{rotations:016d}"
                    put_token(f"{token['value']}\n{new}\n")
                    if stop_rotation.wait(2.5):  # > 2 reload periods (GPUMON_TLS_RELOAD_S=1)
                        break
                    token["value"] = new
                    if stop_rotation.wait(2.5):
                        break
                    put_token(new + "\n")
                    token_rotations += 1

        threading.Thread(target=rotate, daemon=True).start()
    ex = subprocess.Popen(args, env=env, stdout=subprocess.DEVNULL, stderr=open(os.path.join(tmp, "exporter.err"), "wb"))
    windows = []
    probes = probe_failures = metrics_refused = metrics_not_refused = 0
    try:
        deadline = time.monotonic() + 30
        while time.monotonic() < deadline:
            try:
                push_counters(port, ctx, token)
                break
            except (OSError, KeyError, ValueError):
                time.sleep(0.1)
        base = proc_stats(ex.pid)
        end = time.monotonic() + a.minutes * 60
        t0 = time.monotonic()
        while time.monotonic() < end and ex.poll() is None:
            if ctx:
                got, nerr = tls_scrapes(port, ctx, a.window, a.scrape_rate, token)
                r = {"latencies_s": got, "errors": nerr}
            else:
                r = core.scrape_load("127.0.0.1", port, "/metrics", n_requests=0, duration_s=a.window, concurrency=1,
                                     rate_hz=a.scrape_rate, keep_alive=True, gzip=True)
            lat = sorted(r.get("latencies_s", []))
            if a.mtls:
                health, metrics_status = probe_without_cert(port, ctx_nocert)
                probes += len(health)
                probe_failures += sum(1 for st in health if st != 200)
                metrics_refused += metrics_status == 403
                metrics_not_refused += metrics_status != 403
            with sink.lock:
                sk = {"sink_posts": sink.posts, "sink_requests": sink.requests, "sink_handshakes": sink.handshakes,
                      "sink_node_lines": sink.node_lines, "sink_reordered": sink.reordered}
            w = dict(proc_stats(ex.pid), t_min=round((time.monotonic() - t0) / 60, 2), **push_counters(port, ctx, token),
                     **sk, rotations=rotations, token_rotations=token_rotations,
                     scrapes=len(lat), scrape_errors=r.get("errors", 0),
                     scrape_p99_ms=round(lat[int(0.99 * (len(lat) - 1))] * 1e3, 3) if lat else None)
            windows.append(w)
            print(json.dumps(w), flush=True)
    finally:
        stop_rotation.set()
        ex.terminate()
        try:
            ex.wait(timeout=15)
        except subprocess.TimeoutExpired:
            ex.kill()
            ex.wait()
        with open(os.path.join(tmp, "exporter.err"), "rb") as fh:
            err = fh.read()
        if load:
            load.stop()
        sink.shutdown()
        shutil.rmtree(tmp, ignore_errors=True)
    last = windows[-1] if windows else {}
    summary = {
        "minutes": a.minutes, "interval_s": a.interval, "backend": a.backend, "exporter_rc": ex.returncode,
        "windows": len(windows), "ticks": last.get("ticks"),
        "push_ok": last.get("push_ok"), "push_error": last.get("push_error"), "push_dropped": last.get("push_dropped"),
        "sink_posts": last.get("sink_posts"), "sink_requests": last.get("sink_requests"),
        "sink_handshakes": last.get("sink_handshakes"), "sink_reordered": last.get("sink_reordered"),
        "influx_up_end": last.get("influx_up"),
        "fds_start": base.get("fds") if windows else None, "fds_end": last.get("fds"),
        "fds_max": max((w["fds"] for w in windows), default=None),
        "rss_mb_first_window": windows[0]["rss_mb"] if windows else None, "rss_mb_end": last.get("rss_mb"),
        "threads_end": last.get("threads"),
        "scrapes": sum(w["scrapes"] for w in windows), "scrape_errors": sum(w["scrape_errors"] for w in windows),
        "scrape_p99_ms_max_window": max((w["scrape_p99_ms"] or 0 for w in windows), default=None),
        "exporter_stderr_tail": (err or b"").decode(errors="replace")[-400:],
        "close_every": a.close_every, "fail_every": a.fail_every,
        "serve_tls": a.serve_tls, "rotations": rotations, "tls_reloads_ok": last.get("tls_reloads_ok"),
        "tls_reloads_error": last.get("tls_reloads_error"), "tls_handshake_failures": last.get("tls_handshake_failures"),
        "mtls": a.mtls, "probes_without_cert": probes, "probe_failures": probe_failures,
        "metrics_without_cert_403": metrics_refused, "metrics_without_cert_not_403": metrics_not_refused,
        "token": a.token, "token_rotations": token_rotations, "auth_reloads_ok": last.get("auth_reloads_ok"),
        "auth_reloads_error": last.get("auth_reloads_error"), "auth_failures": last.get("auth_failures"),
    }
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
