"""The native gRPC client (csrc/core/grpc_lite.cpp) against a scripted HTTP/2 peer.

The kubelet fixtures (tests/test_native_podresources.py, tests/test_hpack.py) drive the client with
a real grpcio server, which only ever sends well-formed frames. Here a raw unix-socket peer sends
exactly the bytes each case names: padding and PRIORITY fields, CONTINUATION, GOAWAY, RST_STREAM,
a peer that hangs up or never reads, malformed padding, non-200 and Trailers-Only answers, and a
response that never ends. Every case must come back as one named error within the call's deadline;
none may hang the exporter's poller thread (the PodResources and CRI pollers, control_plane.cpp).
The reference has no kubelet client (it shells out to `docker`, /root/reference/gpu.py:177), so
the behaviour pinned here is the framework's own.
"""

import os
import socket
import struct
import threading
import time

import pytest

DATA, HEADERS, RST, SETTINGS, PING, GOAWAY, CONT = 0, 1, 3, 4, 6, 7, 9
END_STREAM, END_HEADERS, PADDED, PRIORITY, ACK = 0x1, 0x4, 0x8, 0x20, 0x1


def frame(typ, flags, stream, payload=b""):
    return struct.pack(">I", len(payload))[1:] + bytes([typ, flags]) + struct.pack(">I", stream) + payload


def lit(name, value):
    """HPACK literal without indexing, plain strings (< 127 bytes)."""
    n, v = name.encode(), value.encode()
    return b"\x00" + bytes([len(n)]) + n + bytes([len(v)]) + v


def msg(body, compressed=False, length=None):
    return bytes([1 if compressed else 0]) + struct.pack(">I", len(body) if length is None else length) + body


def hpack_int(b, i, prefix):
    mask = (1 << prefix) - 1
    v = b[i] & mask
    i += 1
    if v < mask:
        return v, i
    shift = 0
    while True:
        c = b[i]
        i += 1
        v += (c & 0x7F) << shift
        shift += 7
        if not c & 0x80:
            return v, i


def decode_request_headers(block):
    """The client sends 'literal never indexed, new name' fields only (grpc_lite.cpp hpack_literal)."""
    out, i = {}, 0
    while i < len(block):
        assert block[i] == 0x10, block[i]
        n, i = hpack_int(block, i + 1, 7)
        name = block[i:i + n].decode()
        i += n
        n, i = hpack_int(block, i, 7)
        out[name] = block[i:i + n].decode()
        i += n
    return out


OK_HEADERS = frame(HEADERS, END_HEADERS, 1, lit(":status", "200") + lit("content-type", "application/grpc"))
OK_TRAILERS = frame(HEADERS, END_HEADERS | END_STREAM, 1, lit("grpc-status", "0"))


class Peer:
    """One-connection HTTP/2 peer: reads the client's request (unless read=False), then plays
    `script` (bytes to send, "close", or a float to sleep), then holds the connection open."""

    def __init__(self, path, script, read=True):
        self.path, self.script, self.read = path, script, read
        self.request_headers = {}
        self.request_body = b""
        self.frames_after = []  # frames the client sent after its request (SETTINGS/PING ACKs)
        self.stop = threading.Event()
        self.srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.srv.bind(path)
        self.srv.listen(4)
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _recv_frames(self, conn, buf, until):
        while True:
            while len(buf) >= 9:
                n = int.from_bytes(buf[:3], "big")
                if len(buf) < 9 + n:
                    break
                f = (buf[3], buf[4], int.from_bytes(buf[5:9], "big") & 0x7FFFFFFF, bytes(buf[9:9 + n]))
                del buf[:9 + n]
                if until(f):
                    return True
            chunk = conn.recv(1 << 16)
            if not chunk:
                return False
            buf += chunk

    def _run(self):
        conn, _ = self.srv.accept()
        try:
            buf = bytearray()
            if self.read:
                while len(buf) < 24:
                    buf += conn.recv(24 - len(buf))
                assert bytes(buf[:24]) == b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"
                del buf[:24]
                block = bytearray()

                def until(f):
                    typ, flags, stream, pl = f
                    if typ == HEADERS and stream == 1:
                        block.extend(pl)
                    elif typ == DATA and stream == 1:
                        self.request_body += pl
                        return bool(flags & END_STREAM)
                    return False

                self._recv_frames(conn, buf, until)
                self.request_headers = decode_request_headers(bytes(block))
            for step in self.script:
                if step == "close":
                    conn.close()
                    return
                if isinstance(step, float):
                    time.sleep(step)
                else:
                    conn.sendall(step)
            if self.read:
                conn.settimeout(0.5)
                try:
                    self._recv_frames(conn, buf, lambda f: self.frames_after.append(f) and False)
                except OSError:
                    pass
            self.stop.wait(10)
        except OSError:
            pass  # the client hung up first (the error cases)
        finally:
            conn.close()

    def close(self):
        self.stop.set()
        self.srv.close()
        self.t.join(5)


@pytest.fixture
def peer(tmp_path):
    made = []

    def make(script, read=True):
        p = Peer(str(tmp_path / f"h2-{len(made)}.sock"), script, read)
        made.append(p)
        return p

    yield make
    for p in made:
        p.close()


def call(core, p, path="/v1.PodResourcesLister/List", request=b"", timeout_ms=2000):
    t0 = time.monotonic()
    r = core.grpc_call(p.path, path, request, timeout_ms)
    return r, time.monotonic() - t0


def test_padding_priority_and_continuation_are_decoded(core, peer):
    body = b"\x0a\x03abc"
    hdr = lit(":status", "200") + lit("content-type", "application/grpc")
    pad = 7
    # HEADERS with PADDED + PRIORITY (5 bytes of dependency/weight) and no END_HEADERS, then the
    # rest of the block in a CONTINUATION; DATA padded; trailers in their own HEADERS frame.
    first = bytes([pad]) + b"\x00\x00\x00\x00\x10" + hdr[:5] + b"\x00" * pad
    p = peer([frame(SETTINGS, 0, 0), frame(PING, 0, 0, b"12345678"),
              frame(HEADERS, PADDED | PRIORITY, 1, first), frame(CONT, END_HEADERS, 1, hdr[5:]),
              frame(DATA, PADDED, 1, bytes([3]) + msg(body) + b"\x00" * 3), OK_TRAILERS])
    r, _ = call(core, p)
    assert r["ok"], r
    assert r["response"] == body and r["http_status"] == 200 and r["code"] == 0
    # The client acknowledged the peer's SETTINGS and echoed its PING.
    p.t.join(3)
    kinds = {(f[0], f[1]) for f in p.frames_after}
    assert (SETTINGS, ACK) in kinds
    assert any(f[0] == PING and f[1] == ACK and f[3] == b"12345678" for f in p.frames_after)


def test_request_headers_and_long_path(core, peer):
    """A :path of >= 127 bytes takes HPACK's multi-byte integer form (RFC 7541 5.1)."""
    long_path = "/v1." + "x" * 300 + "/List"
    p = peer([OK_HEADERS, frame(DATA, 0, 1, msg(b"")), OK_TRAILERS])
    r, _ = call(core, p, path=long_path, request=b"\x08\x01")
    assert r["ok"], r
    p.t.join(0.1)
    h = p.request_headers
    assert h[":path"] == long_path and h[":method"] == "POST" and h["te"] == "trailers"
    assert h["content-type"] == "application/grpc"
    assert p.request_body == msg(b"\x08\x01")


@pytest.mark.parametrize("script,error", [
    ([frame(GOAWAY, 0, 0, b"\x00\x00\x00\x00\x00\x00\x00\x00")], "GOAWAY from server"),
    ([OK_HEADERS, frame(RST, 0, 1, b"\x00\x00\x00\x02")], "stream reset by server"),
    ([OK_HEADERS, frame(DATA, PADDED, 1)], "bad padded DATA"),
    ([OK_HEADERS, frame(DATA, PADDED, 1, b"\x09abc")], "bad DATA padding"),
    ([frame(HEADERS, PADDED | END_HEADERS, 1)], "bad padded HEADERS"),
    ([frame(HEADERS, PADDED | END_HEADERS, 1, b"\x05ab")], "bad HEADERS padding"),
    ([frame(HEADERS, PRIORITY | END_HEADERS, 1, b"\x00\x00")], "bad HEADERS padding"),
    ([frame(CONT, END_HEADERS, 1, lit(":status", "200"))], "malformed header block sequence"),
    ([frame(HEADERS, 0, 1, lit(":status", "200")), frame(HEADERS, END_HEADERS, 1, b"")],
     "malformed header block sequence"),
    ([frame(HEADERS, END_HEADERS, 1, b"\xff\xff\xff\xff\xff\xff\xff\xff\xff\xff\xff")], "hpack"),
    ([OK_HEADERS, frame(DATA, 0, 1, msg(b"abc")[:4]), "close"], "connection closed"),
    (["close"], "connection closed"),
    ([frame(HEADERS, END_HEADERS | END_STREAM, 1, lit(":status", "503"))], "HTTP :status 503"),
    ([frame(HEADERS, END_HEADERS | END_STREAM, 1, lit(":status", "404") + lit("grpc-status", "12"))],
     "HTTP :status 404, grpc-status 12 UNIMPLEMENTED"),
    ([frame(HEADERS, END_HEADERS | END_STREAM, 1,
            lit(":status", "200") + lit("grpc-status", "7") + lit("grpc-message", "no%20access"))],
     "grpc-status 7 PERMISSION_DENIED: no access"),
    ([OK_HEADERS, OK_TRAILERS], "grpc-status 0 OK without a response message"),
    ([OK_HEADERS, frame(DATA, END_STREAM, 1)], "no gRPC message and no grpc-status in the response"),
    ([OK_HEADERS, frame(DATA, 0, 1, msg(b"abc", compressed=True)), OK_TRAILERS],
     "compressed gRPC message not supported"),
    ([OK_HEADERS, frame(DATA, 0, 1, msg(b"abc", length=10)), OK_TRAILERS], "truncated gRPC message"),
])
def test_malformed_or_failed_responses_name_the_error(core, peer, script, error):
    r, dt = call(core, peer(script))
    assert not r["ok"]
    assert error.lower() in r["error"].lower(), r
    assert dt < 1.5, dt


def test_silent_peer_times_out_at_the_deadline(core, peer):
    p = peer([frame(SETTINGS, 0, 0), OK_HEADERS])  # then nothing
    r, dt = call(core, p, timeout_ms=300)
    assert not r["ok"] and r["error"] == "timeout", r
    assert 0.25 < dt < 1.5, dt


def test_peer_that_never_reads_cannot_stall_the_write(core, peer):
    """An 8 MiB request overflows the unix socket's buffer. A peer that accepts and never reads
    would block a blocking send() forever; the client must give up at its deadline."""
    p = peer([], read=False)
    r, dt = call(core, p, request=b"\x00" * (8 << 20), timeout_ms=300)
    assert not r["ok"] and r["error"] == "write failed", r
    assert dt < 2.0, dt


def test_endless_response_is_capped(core, peer):
    chunk = frame(DATA, 0, 1, b"\x00" * (1 << 20))
    p = peer([OK_HEADERS] + [chunk] * 66)
    r, dt = call(core, p, timeout_ms=10000)
    assert not r["ok"] and r["error"] == "response too large", r
    assert dt < 8, dt


def test_unix_scheme_and_overlong_socket_path(core, peer, tmp_path):
    p = peer([OK_HEADERS, frame(DATA, 0, 1, msg(b"\x08\x01")), OK_TRAILERS])
    r = core.grpc_call("unix://" + p.path, "/v1.PodResourcesLister/List", b"", 2000)
    assert r["ok"] and r["response"] == b"\x08\x01", r
    r = core.grpc_call("/" + "d" * 200 + "/kubelet.sock", "/x", b"", 500)
    assert not r["ok"] and r["error"] == "socket path too long", r
    r = core.grpc_call(str(tmp_path / "absent.sock"), "/x", b"", 500)
    assert not r["ok"] and r["error"].startswith("connect "), r
    assert os.path.exists(p.path)
