"""Synchronizer sheet handling (R7c-R7e, N4): header inference, CSV, row parsing,
authorization filter, quota mapping (reference src/synchronizer.rs:63-286)."""
import json
import shutil
import subprocess

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from bacchus_gpu_controller_amd.testing.fake_google import FORM_HEADERS, make_csv


@pytest.mark.parametrize("header,field", [
    ("타임스탬프", "timestamp"), ("이름", "name"), ("소속", "department"),
    ("SNUCSE ID (id.snucse.org 계정)", "id_username"), ("사용할 서버", "gpu_server"),
    ("GPU 개수", "gpu_request"), ("vCPU 개수", "cpu_request"), ("메모리 (GiB)", "memory_request"),
    ("스토리지 (GiB)", "storage_request"), ("MiG 개수", "mig_request"), ("요청 사유", "description"),
    ("승인", "authorized"), ("이메일 주소", "email"),
])
def test_infer_header(nat, header, field):
    assert nat.infer_header(header) == field


def test_infer_header_exact_vs_substring(nat):
    # exact-match rules: "이름" alone, not as a substring
    with pytest.raises(ValueError, match='unknown header: "실명 이름"'):
        nat.infer_header("실명 이름")
    # substring rules are tested in order: a header mentioning both GPU 개수 and 메모리 -> gpu
    assert nat.infer_header("GPU 개수 / 메모리") == "gpu_request"


def test_unknown_header_fails_whole_parse(nat):
    with pytest.raises(ValueError, match="unknown header"):
        nat.parse_sheet("이름,whatever\nx,y\n")


def test_csv_quoting(nat):
    recs = nat.csv_records('a,"b,c","d""e","multi\nline"\r\n\r\n1,2,3,4')
    assert recs == [["a", "b,c", 'd"e', "multi\nline"], ["1", "2", "3", "4"]]
    with pytest.raises(ValueError):
        nat.csv_records('a,"unterminated')


def test_rows_and_bad_row_skip(nat):
    csv = make_csv([{"id_username": "alice", "gpu": 2, "cpu": 16, "mem": 128}])
    csv += "2026/10/01,x@y,BOB,CSE,bob,mi355x-01,notanumber,1,1,1,0,r,O\r\n"   # bad i64 -> skipped
    csv += "too,few,fields\r\n"                                                  # wrong width -> skipped
    rows, warnings = nat.parse_sheet(csv)
    assert [r["id_username"] for r in rows] == ["alice"]
    assert rows[0]["gpu_request"] == 2 and rows[0]["memory_request"] == 128
    assert len(warnings) == 2 and all("skipping" in w for w in warnings)


def test_missing_column_skips_every_row(nat):
    headers = [h for h in FORM_HEADERS if not h.startswith("MiG")]
    text = ",".join(headers) + "\n" + ",".join(["t", "e", "n", "d", "alice", "s", "1", "1", "1", "1", "r", "O"]) + "\n"
    rows, warnings = nat.parse_sheet(text)
    assert rows == [] and "missing field `mig_request`" in warnings[0]


@pytest.mark.parametrize("value,ok", [
    ("O", True), ("o", True), ("  O \t", True), ("o\t", True), ("X", False), ("", False), ("OO", False), ("0", False),
    # Rust's str::trim strips Unicode White_Space (synchronizer.rs:225-236)
    ("\u00a0O", True), (" O\u00a0", True), ("\u3000o\u2003", True), ("\u0085O\u2029", True),
    ("\u200bO", False),  # zero-width space is not White_Space
    ("\ufeffO", False),  # nor is a byte-order mark
    # to_lowercase maps only O to o: fullwidth and look-alike letters stay unauthorized
    ("\uff4f", False), ("\uff2f", False), ("\u039f", False), ("\u041e", False), ("\u00d8", False),
])
def test_authorized(nat, value, ok):
    assert nat.is_authorized(value) is ok


# Unicode PropList.txt White_Space (what Rust's char::is_whitespace / str::trim use)
WHITE_SPACE = set(map(chr, [*range(0x09, 0x0E), 0x20, 0x85, 0xA0, 0x1680, *range(0x2000, 0x200B), 0x2028, 0x2029,
                            0x202F, 0x205F, 0x3000]))


def rust_trim(s):
    b, e = 0, len(s)
    while b < e and s[b] in WHITE_SPACE:
        b += 1
    while e > b and s[e - 1] in WHITE_SPACE:
        e -= 1
    return s[b:e]


ALPHABET = sorted(WHITE_SPACE) + list("oO0aZ\u00c0\u00de\u00d7\u0130\u0178\u0391\u03a3\u0410\u0401\uff21\uff2f"
                                      "\u200b\ufeff\u001c\u4e00\U0001F600")


@settings(max_examples=400, deadline=None)
@given(st.text(alphabet=ALPHABET, max_size=12))
def test_unicode_trim_matches_rust_semantics(nat, s):
    assert nat.unicode_trim(s.encode()).decode() == rust_trim(s)


@settings(max_examples=400, deadline=None)
@given(st.text(alphabet=ALPHABET, max_size=12))
def test_unicode_lower_matches_full_lowercase_on_covered_scripts(nat, s):
    # Python's str.lower is the full Unicode mapping, like Rust's to_lowercase (final-sigma
    # context aside: Σ is only lowered to σ here, so it is left out of the comparison)
    if "\u03a3" in s:
        return
    assert nat.unicode_lower(s.encode()).decode() == s.lower()


def test_unicode_helpers_keep_invalid_utf8(nat):
    raw = b"\xa0O\xff\xc3"
    assert nat.unicode_lower(raw) == b"\xa0o\xff\xc3"
    assert nat.unicode_trim(b"\xff \xc2\xa0") == b"\xff"


def test_last_authorized_match_and_server_substring(nat):
    csv = make_csv([
        {"id_username": "alice", "gpu": 1, "gpu_server": "mi355x-01"},
        {"id_username": "alice", "gpu": 4, "gpu_server": "mi355x-01"},
        {"id_username": "alice", "gpu": 8, "gpu_server": "mi355x-01", "authorized": "X"},  # not approved
        {"id_username": "alice", "gpu": 7, "gpu_server": "other-server"},                 # other server
        {"id_username": "bob", "gpu": 2, "gpu_server": "mi355x-01, mi355x-02"},
    ])
    assert nat.lookup_row(csv, "mi355x-01", "alice")["gpu_request"] == 4
    assert nat.lookup_row(csv, "mi355x-02", "bob")["gpu_request"] == 2
    assert nat.lookup_row(csv, "mi355x-02", "alice") is None
    assert nat.lookup_row(csv, "", "alice")["gpu_request"] == 7  # "" matches every row


def test_quota_mapping_amd_keys_sorted(nat):
    row = {"id_username": "a", "gpu_request": 2, "cpu_request": 16, "memory_request": 128, "storage_request": 500,
           "mig_request": 1}
    q = nat.quota_spec(row)
    assert q == ('{"hard":{"limits.cpu":"16","limits.memory":"128Gi","requests.amd.com/gpu":"2",'
                 '"requests.amd.com/gpu-partition":"1","requests.cpu":"16","requests.memory":"128Gi",'
                 '"requests.storage":"500Gi"}}')
    q2 = json.loads(nat.quota_spec(row, "amd.com/gpu", "amd.com/cpx_nps1"))["hard"]
    assert q2["requests.amd.com/cpx_nps1"] == "1"
    assert not any("nvidia" in k for k in q2)


def test_google_assertion_verifies(nat):
    from bacchus_gpu_controller_amd.testing.fake_google import FakeGoogle

    fg = FakeGoogle()
    jwt = nat.google_assertion(fg.service_account_json(), "https://www.googleapis.com/auth/drive.readonly", 1_800_000_000)
    h, c, s = jwt.split(".")
    assert nat.rs256_verify(fg.public_key, h + "." + c, nat.base64_decode(s))
    claims = json.loads(nat.base64_decode(c))
    assert claims == {"iss": fg.client_email, "scope": "https://www.googleapis.com/auth/drive.readonly",
                      "aud": "https://oauth2.googleapis.com/token", "exp": 1_800_003_600, "iat": 1_800_000_000}
    assert json.loads(nat.base64_decode(h)) == {"alg": "RS256", "typ": "JWT", "kid": "kid-1"}
    assert not nat.rs256_verify(fg.public_key, h + "." + c + "x", nat.base64_decode(s))


@pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI not available")
def test_google_assertion_verifies_with_openssl_cli(nat, tmp_path):
    """Independent check of the RS256 JWT: `openssl dgst -verify` on the
    signing input, not our own verifier."""
    from bacchus_gpu_controller_amd.testing.fake_google import FakeGoogle

    fg = FakeGoogle()
    jwt = nat.google_assertion(fg.service_account_json(), "https://www.googleapis.com/auth/drive.readonly", 1_800_000_000)
    h, c, s = jwt.split(".")
    (tmp_path / "pub.pem").write_text(fg.public_key)
    (tmp_path / "input").write_bytes((h + "." + c).encode())
    sig = nat.base64_decode(s)
    (tmp_path / "sig").write_bytes(sig if isinstance(sig, bytes) else sig.encode("latin-1"))

    def verify(inp):
        return subprocess.run(["openssl", "dgst", "-sha256", "-verify", str(tmp_path / "pub.pem"), "-signature",
                               str(tmp_path / "sig"), str(inp)], capture_output=True, text=True)
    ok = verify(tmp_path / "input")
    assert ok.returncode == 0 and "Verified OK" in ok.stdout, ok.stdout + ok.stderr
    (tmp_path / "tampered").write_bytes((h + "." + c + "x").encode())
    assert verify(tmp_path / "tampered").returncode != 0
