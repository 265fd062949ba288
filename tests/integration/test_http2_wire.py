"""HTTP/2 wire-level behaviour of the native gRPC server (native/core/http2.cc), driven
frame by frame from a raw unix socket: the cases a well-behaved grpc-go kubelet rarely
produces but the protocol allows — a tiny peer flow-control window, HEADERS split over
CONTINUATION with PADDED/PRIORITY flags, padded DATA, PING, unknown frame types, client
RST_STREAM of a live stream, an interrupted header block and a bad preface."""
import json
import os
import socket
import struct
import time

import pytest

from bacchus_gpu_controller_amd.testing.kubelet import pb

pytestmark = pytest.mark.slow

PREFACE = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"
DATA, HEADERS, PRIORITY, RST, SETTINGS, PUSH, PING, GOAWAY, WINDOW_UPDATE, CONTINUATION = range(10)
END_STREAM, END_HEADERS, PADDED, PRIO = 0x1, 0x4, 0x8, 0x20


def frame(ftype, flags, sid, payload=b""):
    return struct.pack(">I", len(payload))[1:] + bytes([ftype, flags]) + struct.pack(">I", sid) + payload


class RawConn:
    def __init__(self, path, window=65535):
        self.s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.s.settimeout(5)
        self.s.connect(path)
        self.buf = b""
        self.s.sendall(PREFACE + frame(SETTINGS, 0, 0, struct.pack(">HI", 4, window)))

    def _fill(self, n):
        while len(self.buf) < n:
            chunk = self.s.recv(65536)
            if not chunk:
                raise EOFError
            self.buf += chunk

    def read_frame(self):
        self._fill(9)
        n = int.from_bytes(self.buf[:3], "big")
        self._fill(9 + n)
        ftype, flags, sid = self.buf[3], self.buf[4], struct.unpack(">I", self.buf[5:9])[0] & 0x7FFFFFFF
        payload = self.buf[9:9 + n]
        self.buf = self.buf[9 + n:]
        return ftype, flags, sid, payload

    def send(self, data):
        self.s.sendall(data)

    def close(self):
        self.s.close()


def request_headers(nat, method):
    return nat.hpack_encode([(":method", "POST"), (":scheme", "http"), (":path", method),
                             (":authority", "localhost"), ("content-type", "application/grpc"), ("te", "trailers")])


def grpc_msg(b):
    return b"\x00" + struct.pack(">I", len(b)) + b


def collect_response(conn, nat, sid, replenish=False):
    """Reads until END_STREAM on `sid`; returns (headers, data, trailers, DATA frame sizes)."""
    dec = nat.HpackDecoder()
    headers, trailers, data, sizes = None, None, b"", []
    while True:
        ftype, flags, fsid, payload = conn.read_frame()
        if ftype == SETTINGS and not flags & 1:
            conn.send(frame(SETTINGS, 1, 0))
            continue
        if fsid != sid:
            continue
        if ftype == HEADERS:
            hl = dec.decode(payload)
            if headers is None:
                headers = hl
            else:
                trailers = hl
        elif ftype == DATA:
            data += payload
            sizes.append(len(payload))
            if replenish and payload:
                inc = struct.pack(">I", len(payload))
                conn.send(frame(WINDOW_UPDATE, 0, 0, inc) + frame(WINDOW_UPDATE, 0, sid, inc))
        if flags & END_STREAM:
            return headers, data, trailers, sizes


@pytest.fixture
def plugin(nat, tmp_path):
    d = str(tmp_path / "dp")
    os.makedirs(d)
    p = nat.DevicePlugin(nat.default_mi355x_fixture(8), {"plugin_dir": d, "register": "false"})
    p.start()
    yield p
    p.stop()


def test_tiny_peer_window_is_honoured(nat, plugin):
    c = RawConn(plugin.socket_path, window=10)
    try:
        c.send(frame(HEADERS, END_HEADERS, 1, request_headers(nat, "/v1beta1.DevicePlugin/GetPreferredAllocation")))
        q = pb["PreferredAllocationRequest"]()
        r = q.container_requests.add()
        r.available_deviceIDs.extend([f"dev-{i:04d}" for i in range(200)])
        r.allocation_size = 200
        c.send(frame(DATA, END_STREAM, 1, grpc_msg(q.SerializeToString())))
        headers, data, trailers, sizes = collect_response(c, nat, 1, replenish=True)
        assert (b":status", b"200") in headers and (b"grpc-status", b"0") in trailers
        assert max(sizes) <= 10  # never more than the window we granted
        resp = pb["PreferredAllocationResponse"].FromString(data[5:])
        assert len(resp.container_responses[0].deviceIDs) == 200
    finally:
        c.close()


def test_continuation_padding_priority_ping_and_unknown_frames(nat, plugin):
    c = RawConn(plugin.socket_path)
    try:
        c.send(frame(0x42, 0, 0, b"unknown frame types are ignored"))
        c.send(frame(PING, 0, 0, b"12345678"))
        block = request_headers(nat, "/v1beta1.DevicePlugin/GetDevicePluginOptions")
        # HEADERS (PADDED + PRIORITY) with half the block, CONTINUATION with the rest
        first = bytes([3]) + struct.pack(">IB", 0, 15) + block[:10] + b"\x00" * 3
        c.send(frame(HEADERS, PADDED | PRIO, 1, first))
        c.send(frame(CONTINUATION, END_HEADERS, 1, block[10:]))
        c.send(frame(DATA, PADDED | END_STREAM, 1, bytes([5]) + grpc_msg(b"") + b"\x00" * 5))
        got_ping = False
        dec = nat.HpackDecoder()
        trailers, data = None, b""
        while trailers is None:
            ftype, flags, sid, payload = c.read_frame()
            if ftype == PING and flags & 1:
                assert payload == b"12345678"
                got_ping = True
            elif ftype == HEADERS and sid == 1:
                hl = dec.decode(payload)
                if flags & END_STREAM:
                    trailers = hl
            elif ftype == DATA and sid == 1:
                data += payload
        assert got_ping and (b"grpc-status", b"0") in trailers
        assert pb["DevicePluginOptions"].FromString(data[5:]).get_preferred_allocation_available
    finally:
        c.close()


def test_interrupted_header_block_is_a_connection_error(nat, plugin):
    c = RawConn(plugin.socket_path)
    try:
        block = request_headers(nat, "/v1beta1.DevicePlugin/GetDevicePluginOptions")
        c.send(frame(HEADERS, 0, 1, block[:10]))  # no END_HEADERS ...
        c.send(frame(PING, 0, 0, b"abcdefgh"))  # ... then a non-CONTINUATION frame
        with pytest.raises((EOFError, ConnectionResetError)):
            while True:
                ftype, flags, sid, payload = c.read_frame()
                if ftype == GOAWAY:
                    assert struct.unpack(">I", payload[4:8])[0] == 1  # PROTOCOL_ERROR
    finally:
        c.close()
    # the server keeps serving other connections
    c = RawConn(plugin.socket_path)
    try:
        c.send(frame(HEADERS, END_HEADERS, 1, request_headers(nat, "/v1beta1.DevicePlugin/GetDevicePluginOptions")))
        c.send(frame(DATA, END_STREAM, 1, grpc_msg(b"")))
        _, _, trailers, _ = collect_response(c, nat, 1)
        assert (b"grpc-status", b"0") in trailers
    finally:
        c.close()


def test_unknown_method_is_trailers_only_unimplemented(nat, plugin):
    c = RawConn(plugin.socket_path)
    try:
        c.send(frame(HEADERS, END_HEADERS, 1, request_headers(nat, "/v1beta1.DevicePlugin/Nope")))
        c.send(frame(DATA, END_STREAM, 1, grpc_msg(b"")))
        headers, data, trailers, _ = collect_response(c, nat, 1)
        assert trailers is None and data == b""  # trailers-only response
        assert (b"grpc-status", b"12") in headers
    finally:
        c.close()


def test_client_reset_ends_list_and_watch(nat, plugin):
    c = RawConn(plugin.socket_path)
    try:
        c.send(frame(HEADERS, END_HEADERS, 1, request_headers(nat, "/v1beta1.DevicePlugin/ListAndWatch")))
        c.send(frame(DATA, END_STREAM, 1, grpc_msg(b"")))
        dec = nat.HpackDecoder()
        while True:  # the first device list arrives
            ftype, flags, sid, payload = c.read_frame()
            if ftype == HEADERS and sid == 1:
                dec.decode(payload)
            if ftype == DATA and sid == 1:
                assert len(pb["ListAndWatchResponse"].FromString(payload[5:]).devices) == 8
                break
        c.send(frame(RST, 0, 1, struct.pack(">I", 8)))  # CANCEL
        # a health flip after the reset is not written to the cancelled stream, and the
        # connection stays usable for new calls.  (Give the server a moment to read the
        # RST_STREAM first: a flip racing it may legally still be in flight.)
        time.sleep(0.2)
        plugin.set_health([False] + [True] * 7)
        time.sleep(0.3)
        c.send(frame(HEADERS, END_HEADERS, 3, request_headers(nat, "/v1beta1.DevicePlugin/GetDevicePluginOptions")))
        c.send(frame(DATA, END_STREAM, 3, grpc_msg(b"")))
        while True:
            ftype, flags, sid, payload = c.read_frame()
            assert not (sid == 1 and ftype == DATA), "data on a reset stream"
            if sid == 3 and ftype == HEADERS and flags & END_STREAM:
                break
    finally:
        c.close()
    assert json.loads(plugin.describe())["devices"][0]["health"] == "Unhealthy"


def test_bad_preface_closes_connection(plugin):
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.settimeout(5)
    s.connect(plugin.socket_path)
    s.sendall(b"GET / HTTP/1.1\r\nHost: x\r\n\r\n")
    got = b""
    try:
        while True:
            chunk = s.recv(4096)
            if not chunk:
                break
            got += chunk
    except (ConnectionResetError, socket.timeout):
        pass
    s.close()
    assert b"HTTP/1.1 200" not in got
