"""The native HTTP stack (native/core/http.cc, http2.cc, net.cc) end to end through its
pybind surface: a TLS test server and the native client, over HTTP/1.1 and HTTP/2 (ALPN).

What the services rely on: multiplexed concurrent requests; flow control both ways for
bodies larger than a window; streamed responses; graceful drain on stop (GOAWAY, requests
in flight finish); reconnect after the server idles a connection out; a timed-out stream
reset without losing the connection; and HTTP/1.1 fallback when the server does not offer h2.
The client side runs in both HTTP/2 modes: a reader thread per connection, and caller-reads.
"""
import threading
import time

import pytest


@pytest.fixture(scope="module")
def pki(nat):
    return nat.make_ca_and_leaf("http-test", ["localhost", "127.0.0.1"], 1, "ec")


@pytest.fixture
def server(nat, pki):
    s = nat.HttpTestServer(pki["cert"], pki["key"])
    yield s
    s.stop(0)


_MODE = {"caller_reads": False}


@pytest.fixture(autouse=True, params=[False, True], ids=["reader-thread", "caller-reads"])
def h2_client_mode(request):
    """Every test runs twice: HTTP/2 client connections with their own reader thread, and
    in caller-reads mode (the waiting callers read the frames; kube-lite's webhook client)."""
    _MODE["caller_reads"] = request.param
    yield request.param


def client(nat, pki, port, **kw):
    kw.setdefault("h2_caller_reads", _MODE["caller_reads"])
    return nat.HttpClient(f"https://127.0.0.1:{port}", pki["ca_cert"], **kw)


@pytest.mark.parametrize("http2", [True, False])
def test_echo_negotiates_protocol(nat, pki, server, http2):
    c = client(nat, pki, server.port, http2=http2)
    status, body, headers = c.request("POST", "/echo?a=1&b=2", b"hello")
    assert (status, body) == (200, b"hello")
    assert headers["x-protocol"] == ("HTTP/2" if http2 else "HTTP/1.1")
    assert headers["x-echo-query"] == "a=1&b=2"
    assert headers["content-type"] == "application/octet-stream"


def test_h2_falls_back_to_http11_when_server_offers_no_h2(nat, pki):
    s = nat.HttpTestServer(pki["cert"], pki["key"], http2=False)
    try:
        c = client(nat, pki, s.port, http2=True)
        for _ in range(3):
            status, _, headers = c.request("POST", "/echo", b"x")
            assert status == 200 and headers["x-protocol"] == "HTTP/1.1"
    finally:
        s.stop(0)


def test_h2_bodies_larger_than_flow_control_windows(nat, pki, server):
    c = client(nat, pki, server.port)
    big = bytes(range(256)) * (5 * 4096)  # 5 MiB up: > 1 MiB stream window
    status, body, headers = c.request("POST", "/echo", big)
    assert status == 200 and body == big and headers["x-protocol"] == "HTTP/2"
    status, body, _ = c.request("GET", f"/big?n={3 << 20}")  # 3 MiB down: > 64 KiB default peer window
    assert status == 200 and len(body) == 3 << 20 and body[4096:4097] == b"b"


def test_h2_many_concurrent_requests_one_connection(nat, pki, server):
    c = client(nat, pki, server.port)
    errors, done = [], []

    def worker(k):
        try:
            for i in range(20):
                payload = f"{k}-{i}".encode() * 50
                status, body, _ = c.request("POST", f"/echo?k={k}", payload)
                assert status == 200 and body == payload
            done.append(k)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(32)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not errors and len(done) == 32


def test_h2_streamed_response(nat, pki, server):
    c = client(nat, pki, server.port)
    status, body, _ = c.request("GET", "/chunks?n=50")
    lines = body.decode().splitlines()
    assert status == 200 and lines[0] == '{"i":0}' and lines[-1] == '{"i":49}' and len(lines) == 50


def test_h2_timeout_resets_only_the_stream(nat, pki, server):
    c = client(nat, pki, server.port)
    assert c.request("POST", "/echo", b"warm")[0] == 200
    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match="timeout"):
        c.request("GET", "/slow?ms=1500", timeout_ms=200)
    assert time.monotonic() - t0 < 1.2
    # the connection (and its other streams) is still good
    assert c.request("POST", "/echo", b"after")[1] == b"after"


@pytest.mark.parametrize("http2", [True, False])
def test_graceful_stop_finishes_requests_in_flight(nat, pki, http2):
    s = nat.HttpTestServer(pki["cert"], pki["key"])
    c = client(nat, pki, s.port, http2=http2)
    assert c.request("POST", "/echo", b"x")[0] == 200  # connection established
    out = {}

    def slow():
        try:
            out["r"] = c.request("GET", "/slow?ms=600")
        except Exception as e:  # noqa: BLE001
            out["e"] = repr(e)

    t = threading.Thread(target=slow)
    t.start()
    time.sleep(0.2)
    t0 = time.monotonic()
    s.stop(5000)  # drains: GOAWAY over h2, then waits for the stream in flight
    t.join(10)
    assert out.get("r", (None, None))[:2] == (200, b"done"), out
    assert time.monotonic() - t0 < 4


def test_client_reconnects_after_server_idles_connection_out(nat, pki):
    s = nat.HttpTestServer(pki["cert"], pki["key"], idle_timeout_ms=300)
    try:
        c = client(nat, pki, s.port)
        assert c.request("POST", "/echo", b"1")[0] == 200
        time.sleep(1.2)  # the server closes the idle h2 connection (GOAWAY + close)
        status, body, headers = c.request("POST", "/echo", b"2")
        assert (status, body, headers["x-protocol"]) == (200, b"2", "HTTP/2")
    finally:
        s.stop(0)


def test_h2_spreads_over_several_connections(nat, pki, server):
    c = client(nat, pki, server.port, h2_connections=3)
    for i in range(9):
        assert c.request("POST", "/echo", str(i).encode())[1] == str(i).encode()
    assert server.served >= 9


def test_h2_inline_handlers(nat, pki):
    """h2_inline_paths: a stream that arrives on an idle connection runs on the reader
    thread.  Streams that arrive while another is in flight still go to workers, and a
    response larger than the client's 64 KiB window is finished on a worker: the reader
    thread cannot wait for a WINDOW_UPDATE that only it can read."""
    s = nat.HttpTestServer(pki["cert"], pki["key"], inline_paths=["/echo", "/big", "/slow"])
    try:
        c = client(nat, pki, s.port)
        for i in range(5):
            assert c.request("POST", "/echo", str(i).encode())[1] == str(i).encode()
        assert s.inline_served == 5
        # 3 MiB down through the blocked-send hand-off, twice (the connection stays good)
        for _ in range(2):
            status, body, _ = c.request("GET", f"/big?n={3 << 20}")
            assert status == 200 and len(body) == 3 << 20 and body[4096:4097] == b"b"
        # a slow inline handler holds the reader; a concurrent stream waits for it and is
        # then served (on a worker or inline), never lost
        out = {}
        t = threading.Thread(target=lambda: out.setdefault("slow", c.request("GET", "/slow?ms=300")))
        t.start()
        time.sleep(0.05)
        assert c.request("POST", "/echo", b"during")[1] == b"during"
        t.join(10)
        assert out["slow"][:2] == (200, b"done")
    finally:
        s.stop(0)


def test_h2_inline_concurrent_streams_one_connection(nat, pki):
    s = nat.HttpTestServer(pki["cert"], pki["key"], inline_paths=["/echo"])
    try:
        c = client(nat, pki, s.port)
        errors = []

        def worker(k):
            try:
                for i in range(30):
                    payload = f"{k}-{i}".encode() * 40
                    status, body, _ = c.request("POST", "/echo", payload)
                    assert status == 200 and body == payload
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))

        ts = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(60)
        assert not errors
        assert s.served == 16 * 30 and 0 < s.inline_served <= s.served
    finally:
        s.stop(0)


def test_a_timed_out_request_drops_the_pooled_connections():
    """Round 5: a request that gets no answer within its timeout means the path to the
    server may be dead, and every pooled connection with it (a wedged proxy, an expired NAT
    entry).  The client drops them all instead of trying the next one, so the request after
    the failure dials afresh and succeeds at once."""
    import http.server
    import threading
    import time

    from bacchus_gpu_controller_amd import native
    from bacchus_gpu_controller_amd.testing.stall_proxy import StallProxy

    class H(http.server.BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def do_GET(self):
            time.sleep(0.05)  # keeps concurrent requests on separate connections
            self.send_response(200)
            self.send_header("Content-Length", "2")
            self.end_headers()
            self.wfile.write(b"ok")

        def log_message(self, *a):
            pass

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    proxy = StallProxy("127.0.0.1", srv.server_address[1]).start()
    try:
        c = native().HttpClient(proxy.url, http2=False, timeout_ms=300)
        ts = [threading.Thread(target=lambda: c.request("GET", "/")) for _ in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert proxy.accepted >= 3  # several keep-alive connections in the pool
        proxy.freeze()
        t0 = time.monotonic()
        with pytest.raises(RuntimeError, match="timeout"):
            c.request("GET", "/")
        assert time.monotonic() - t0 < 0.6  # one timeout, not one per pooled connection
        before = proxy.accepted
        t0 = time.monotonic()
        assert c.request("GET", "/")[0] == 200
        assert time.monotonic() - t0 < 0.25 and proxy.accepted == before + 1
    finally:
        proxy.stop()
        srv.shutdown()


def test_a_stale_pooled_connection_is_retried_on_a_fresh_one():
    """A server that closes idle connections (an idle timeout) may close a pooled one just
    as the client sends on it, and usually closes the connections opened with it too.  The
    client's one retry of an unanswered request therefore dials afresh instead of taking the
    next pooled connection (which would fail the same way)."""
    import socket
    import threading
    import time

    from bacchus_gpu_controller_amd import native

    lsock = socket.socket()
    lsock.bind(("127.0.0.1", 0))
    lsock.listen(16)
    accepted = []

    def serve(conn):
        buf, served = b"", 0
        while True:
            while b"\r\n\r\n" not in buf:
                d = conn.recv(4096)
                if not d:
                    conn.close()
                    return
                buf += d
            buf = buf.split(b"\r\n\r\n", 1)[1]
            if served == 1:  # the server's idle close, racing the client's second request
                conn.close()
                return
            time.sleep(0.05)  # keeps the first, concurrent requests on separate connections
            conn.sendall(b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\nok")
            served += 1

    def accept_loop():
        while True:
            try:
                conn, _ = lsock.accept()
            except OSError:
                return
            accepted.append(conn)
            threading.Thread(target=serve, args=(conn,), daemon=True).start()

    threading.Thread(target=accept_loop, daemon=True).start()
    try:
        c = native().HttpClient(f"http://127.0.0.1:{lsock.getsockname()[1]}", http2=False, timeout_ms=2000)
        ts = [threading.Thread(target=lambda: c.request("GET", "/")) for _ in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert len(accepted) == 2  # two pooled keep-alive connections, both about to fail
        assert c.request("GET", "/")[0] == 200
        assert len(accepted) == 3  # the retry dialled a new connection
    finally:
        lsock.close()
