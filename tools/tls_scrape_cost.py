#!/usr/bin/env python3
"""What serving /metrics over HTTPS costs: the exporter's own service time per scrape (request parsed
-> last byte written, Exporter.scrape_durations_since) and the client's round trip. Plain HTTP is
compared with TLS, identity with gzip, on a mock 8-GPU exposition. One keep-alive connection
scrapes back to back, as Prometheus does, so the TLS handshake is paid once. Prints one JSON line
per shape.
"""

import argparse
import http.client
import json
import os
import ssl
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _pct(v, q):
    v = sorted(v)
    return round(v[min(len(v) - 1, int(q * (len(v) - 1)))] * 1e3, 4) if v else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--gpus", type=int, default=8)
    a = ap.parse_args()
    from gpumon import core as _core

    c = _core()
    with tempfile.TemporaryDirectory() as d:
        subprocess.run(["openssl", "req", "-x509", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1",
                        "-nodes", "-days", "1", "-keyout", f"{d}/k.pem", "-out", f"{d}/c.pem", "-subj", "/CN=localhost",
                        "-addext", "subjectAltName=DNS:localhost"], check=True, capture_output=True, timeout=60)
        for tls in (False, True):
            cfg = {"backend": f"mock:gpus={a.gpus}", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                   "http_threads": 1, "host": "node"}
            if tls:
                cfg.update(tls_cert_file=f"{d}/c.pem", tls_key_file=f"{d}/k.pem")
            ex = c.Exporter(cfg)
            ex.start()
            ex.tick()
            for gz in (False, True):
                ctx = ssl.create_default_context(cafile=f"{d}/c.pem") if tls else None
                conn = (http.client.HTTPSConnection("localhost", ex.port, context=ctx, timeout=5) if tls
                        else http.client.HTTPConnection("127.0.0.1", ex.port, timeout=5))
                hdr = {"Accept-Encoding": "gzip"} if gz else {}
                t_hs = time.perf_counter()
                conn.request("GET", "/metrics", headers=hdr)
                body = conn.getresponse().read()
                first_ms = (time.perf_counter() - t_hs) * 1e3  # includes the handshake on TLS
                n0 = ex.scrape_count()
                client = []
                for _ in range(a.n):
                    t = time.perf_counter()
                    conn.request("GET", "/metrics", headers=hdr)
                    conn.getresponse().read()
                    client.append(time.perf_counter() - t)
                conn.close()
                time.sleep(0.05)
                srv = list(ex.scrape_durations_since(n0))
                print(json.dumps({"tls": tls, "gzip": gz, "gpus": a.gpus, "body_kb": round(len(body) / 1024, 1),
                                  "scrapes": len(client), "first_request_ms": round(first_ms, 3),
                                  "server_p50_ms": _pct(srv, 0.5), "server_p99_ms": _pct(srv, 0.99),
                                  "client_p50_ms": _pct(client, 0.5), "client_p99_ms": _pct(client, 0.99)}), flush=True)
            ex.stop()


if __name__ == "__main__":
    main()
