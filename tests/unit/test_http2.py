"""HPACK/Huffman, protobuf wire codecs and the xGMI-aware allocation policy behind the
native kubelet device plugin (native/core/{hpack,protobuf}.cc, native/gpu/device_plugin.cc).

Independent oracles: libnghttp2 (system library, via ctypes) for HPACK, python protobuf
(dynamic descriptors of the v1beta1 API) for the message layouts."""
import ctypes
import ctypes.util
import json
import random
from fractions import Fraction

import pytest

from bacchus_gpu_controller_amd.testing.kubelet import pb


def _nghttp2():
    for name in ("libnghttp2.so.14", ctypes.util.find_library("nghttp2")):
        if not name:
            continue
        try:
            return ctypes.CDLL(name)
        except OSError:
            continue
    pytest.skip("libnghttp2 not available")


class _NV(ctypes.Structure):
    _fields_ = [("name", ctypes.c_void_p), ("value", ctypes.c_void_p), ("namelen", ctypes.c_size_t),
                ("valuelen", ctypes.c_size_t), ("flags", ctypes.c_uint8)]


class Nghttp2Hpack:
    """Thin ctypes wrapper over nghttp2's public HPACK inflater/deflater."""

    def __init__(self):
        self.lib = lib = _nghttp2()
        lib.nghttp2_hd_inflate_hd2.restype = ctypes.c_ssize_t
        lib.nghttp2_hd_inflate_hd2.argtypes = [ctypes.c_void_p, ctypes.POINTER(_NV), ctypes.POINTER(ctypes.c_int),
                                               ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
        lib.nghttp2_hd_deflate_hd.restype = ctypes.c_ssize_t
        lib.nghttp2_hd_deflate_hd.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(_NV),
                                              ctypes.c_size_t]
        lib.nghttp2_hd_deflate_bound.restype = ctypes.c_size_t
        lib.nghttp2_hd_deflate_bound.argtypes = [ctypes.c_void_p, ctypes.POINTER(_NV), ctypes.c_size_t]
        self.inf = ctypes.c_void_p()
        assert lib.nghttp2_hd_inflate_new(ctypes.byref(self.inf)) == 0
        self.dfl = ctypes.c_void_p()
        assert lib.nghttp2_hd_deflate_new(ctypes.byref(self.dfl), ctypes.c_size_t(4096)) == 0

    def inflate(self, block):
        out, buf = [], ctypes.create_string_buffer(block, len(block))
        off = 0
        while True:
            nv, fl = _NV(), ctypes.c_int(0)
            rv = self.lib.nghttp2_hd_inflate_hd2(self.inf, ctypes.byref(nv), ctypes.byref(fl),
                                                 ctypes.cast(ctypes.addressof(buf) + off, ctypes.c_char_p),
                                                 len(block) - off, 1)
            assert rv >= 0, f"nghttp2 inflate error {rv}"
            off += rv
            if fl.value & 0x02:  # EMIT
                out.append((ctypes.string_at(nv.name, nv.namelen), ctypes.string_at(nv.value, nv.valuelen)))
            if fl.value & 0x01:  # FINAL
                self.lib.nghttp2_hd_inflate_end_headers(self.inf)
                return out
            if not (fl.value & 0x02) and off >= len(block):
                return out

    def deflate(self, headers):
        keep = []
        arr = (_NV * len(headers))()
        for i, (k, v) in enumerate(headers):
            kb, vb = ctypes.create_string_buffer(k, len(k)), ctypes.create_string_buffer(v, len(v))
            keep += [kb, vb]
            arr[i] = _NV(ctypes.addressof(kb), ctypes.addressof(vb), len(k), len(v), 0)
        bound = self.lib.nghttp2_hd_deflate_bound(self.dfl, arr, len(headers))
        out = ctypes.create_string_buffer(bound)
        n = self.lib.nghttp2_hd_deflate_hd(self.dfl, out, bound, arr, len(headers))
        assert n >= 0
        return out.raw[:n]


def _hpack_int(v, prefix, first):
    mask = (1 << prefix) - 1
    if v < mask:
        return bytes([first | v])
    out = [first | mask]
    v -= mask
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def test_huffman_every_byte_decodes_in_nghttp2(nat):
    """Our Huffman table (RFC 7541 App. B) encodes all 256 byte values the way nghttp2 reads them."""
    hp = Nghttp2Hpack()
    rng = random.Random(7)
    for b in range(256):
        value = bytes([b]) + bytes(rng.randrange(256) for _ in range(5)) + bytes([b])
        huff = nat.huffman_encode(value)
        # literal without indexing, new name (raw), Huffman-coded value
        block = b"\x00" + _hpack_int(6, 7, 0) + b"x-byte" + _hpack_int(len(huff), 7, 0x80) + huff
        assert hp.inflate(block) == [(b"x-byte", value)], b
        assert nat.huffman_decode(huff) == value


def test_huffman_table_is_canonical_and_complete(nat):
    # Kraft sum of a complete prefix code is exactly 1; derive lengths from single-symbol encodes.
    lengths = []
    for b in range(256):
        enc = nat.huffman_encode(bytes([b]) * 8)  # 8 copies: total bits = 8*len, no padding
        lengths.append(len(enc))  # == code length in bits
    kraft = sum(Fraction(1, 2 ** n) for n in lengths) + Fraction(1, 2 ** 30)  # + EOS (30 bits)
    assert kraft == 1
    assert lengths[ord("0")] == 5 and lengths[ord("a")] == 5 and lengths[0] == 13 and lengths[255] == 26


def test_huffman_rejects_bad_padding(nat):
    assert nat.huffman_decode(b"\x1f") is not None  # 'a' (00011) + 111 padding
    assert nat.huffman_decode(b"\x18") is None      # 'a' + 000 padding: not an EOS prefix
    assert nat.huffman_decode(b"\xff\xff\xff\xff") is None  # EOS inside the string


def test_hpack_decoder_follows_nghttp2_dynamic_table(nat):
    """nghttp2's deflater indexes incrementally and Huffman-codes; our decoder tracks its table."""
    hp = Nghttp2Hpack()
    dec = nat.HpackDecoder()
    blocks = [
        [(b":method", b"POST"), (b":scheme", b"http"), (b":path", b"/v1beta1.DevicePlugin/Allocate"),
         (b":authority", b"localhost"), (b"content-type", b"application/grpc"), (b"te", b"trailers"),
         (b"user-agent", b"grpc-go/1.65.0")],
        [(b":method", b"POST"), (b":scheme", b"http"), (b":path", b"/v1beta1.DevicePlugin/ListAndWatch"),
         (b":authority", b"localhost"), (b"content-type", b"application/grpc"), (b"te", b"trailers"),
         (b"user-agent", b"grpc-go/1.65.0"), (b"grpc-timeout", b"9999859u")],
        [(b":status", b"200"), (b"content-type", b"application/grpc"), (b"x-bin", bytes(range(256)))],
    ]
    for _ in range(3):
        for hl in blocks:
            assert dec.decode(hp.deflate(hl)) == hl
    assert dec.table_entries > 0


def test_hpack_encoder_roundtrips_through_nghttp2(nat):
    hp = Nghttp2Hpack()
    hl = [(":status", "200"), ("content-type", "application/grpc"), ("grpc-status", "0"),
          ("grpc-message", "unknown device id 0000:ff:00.0"), (":path", "/"), ("x-long", "v" * 300)]
    out = hp.inflate(nat.hpack_encode(hl))
    assert out == [(k.encode(), v.encode()) for k, v in hl]


def test_hpack_decoder_rejects_garbage(nat):
    dec = nat.HpackDecoder()
    with pytest.raises(RuntimeError):
        dec.decode(b"\xff\xff\xff\xff\x7f")  # index overflow / out of range
    with pytest.raises(RuntimeError):
        nat.HpackDecoder().decode(bytes([0x80 | 70]))  # dynamic index on an empty table


# ---------------------------------------------------------------- protobuf layouts
def test_register_request_matches_protobuf(nat):
    req = {"version": "v1beta1", "endpoint": "bgc-amd-gpu.sock", "resource_name": "amd.com/gpu",
           "pre_start_required": False, "get_preferred_allocation_available": True}
    m = pb["RegisterRequest"].FromString(nat.dp_encode("register_request", json.dumps(req)))
    assert (m.version, m.endpoint, m.resource_name) == ("v1beta1", "bgc-amd-gpu.sock", "amd.com/gpu")
    assert m.options.get_preferred_allocation_available and not m.options.pre_start_required
    assert json.loads(nat.dp_decode("register_request", m.SerializeToString())) == req


def test_allocate_and_preferred_messages_match_protobuf(nat):
    r = pb["AllocateRequest"]()
    r.container_requests.add().devices_ids.extend(["0000:05:00.0", "0000:15:00.0"])
    r.container_requests.add().devices_ids.extend(["0000:75:00.0"])
    assert json.loads(nat.dp_decode("allocate_request", r.SerializeToString())) == [
        ["0000:05:00.0", "0000:15:00.0"], ["0000:75:00.0"]]
    q = pb["PreferredAllocationRequest"]()
    c = q.container_requests.add()
    c.available_deviceIDs.extend(["a", "b", "c"])
    c.must_include_deviceIDs.append("b")
    c.allocation_size = 2
    assert json.loads(nat.dp_decode("preferred_request", q.SerializeToString())) == [
        {"available": ["a", "b", "c"], "must_include": ["b"], "size": 2}]
    resp = pb["PreferredAllocationResponse"].FromString(nat.dp_encode("preferred_response", json.dumps([["b", "a"]])))
    assert list(resp.container_responses[0].deviceIDs) == ["b", "a"]
    # a message with an unknown field (newer kubelet) still decodes
    raw = r.SerializeToString() + b"\xa2\x06\x03xyz"  # field 100, length-delimited
    assert len(json.loads(nat.dp_decode("allocate_request", raw))) == 2


def test_list_and_watch_numa_zero_is_present(nat):
    devs = [{"id": "g0", "healthy": True, "numa_nodes": [0]}, {"id": "g1", "healthy": False, "numa_nodes": [1]}]
    m = pb["ListAndWatchResponse"].FromString(nat.dp_encode("list_and_watch", json.dumps(devs)))
    assert [(d.ID, d.health, [n.ID for n in d.topology.nodes]) for d in m.devices] == [
        ("g0", "Healthy", [0]), ("g1", "Unhealthy", [1])]


# ---------------------------------------------------------------- allocation policy
def _two_hives(nat):
    a = json.loads(nat.default_mi355x_fixture(8, 0xAAAA))["gpus"]
    b = json.loads(nat.default_mi355x_fixture(4, 0xBBBB))["gpus"]
    for i, g in enumerate(b):
        g["index"] = 8 + i
        g["bdf"] = f"0000:{0x85 + 0x10 * i:02x}:00.0"
        g["numa_node"] = 1
    gpus = a + b
    return gpus, [g["bdf"] for g in gpus]


def test_preferred_allocation_packs_one_hive_best_fit(nat):
    gpus, ids = _two_hives(nat)
    js = json.dumps(gpus)
    # 4 GPUs fit both hives: best fit picks the 4-GPU hive and keeps the 8-GPU island whole for TP=8
    got = nat.preferred_allocation(js, ids, ids, [], 4)
    assert sorted(got) == sorted(ids[8:])
    # 8 GPUs: only the big hive holds them
    got = nat.preferred_allocation(js, ids, ids, [], 8)
    assert sorted(got) == sorted(ids[:8])
    # must-include pulls the allocation into its hive and NUMA node
    got = nat.preferred_allocation(js, ids, ids, [ids[5]], 3)
    assert got[0] == ids[5] and all(g in ids[4:8] for g in got)
    # 2 GPUs inside the 8-hive when the small hive is busy: same NUMA, adjacent xGMI nodes
    got = nat.preferred_allocation(js, ids, ids[:8], [], 2)
    assert got == [ids[0], ids[1]]


def test_preferred_allocation_spans_fewest_hives(nat):
    gpus, ids = _two_hives(nat)
    avail = ids[:3] + ids[8:]  # 3 left on hive A, 4 on hive B
    got = nat.preferred_allocation(json.dumps(gpus), ids, avail, [], 6)
    assert len(got) == 6 and set(ids[8:]) <= set(got)  # the whole bigger remainder first


def test_preferred_allocation_ignores_duplicate_ids(nat):
    gpus, ids = _two_hives(nat)
    got = nat.preferred_allocation(json.dumps(gpus), ids, ids[:2] * 3 + ids[2:4], [ids[0]], 3)
    assert len(got) == len(set(got)) == 3 and got[0] == ids[0]
