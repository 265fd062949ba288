"""Fake Google OAuth2 token endpoint + Drive v3 export (north-star N7, "fake Google").

* ``POST /token``: JWT-bearer grant. The RS256 assertion is verified against the
  service account's public key with the native verifier, and its claims (iss, aud,
  scope, exp) are checked — so the synchronizer's hand-rolled service-account flow is
  tested end to end, not mocked.
* ``GET /drive/v3/files/<id>/export?mimeType=text/csv``: returns the current CSV for a
  valid bearer token.
* ``GET /drive/v3/files/<id>?fields=version``: file metadata; ``version`` goes up on every
  sheet edit, like Drive's.
* ``POST /_fake/rows`` ``{"rows": [...], "append": bool}``: edit the sheet over HTTP (the
  operator approving rows; used by bench ranks that do not own this object).
* Fault knobs: ``fail_export`` / ``fail_token`` (HTTP status to return), ``export_delay``.
"""
import json
import threading
import time
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from .. import native

SCOPE = "https://www.googleapis.com/auth/drive.readonly"

# Header row of the Korean Google Form (order as exported; reference
# src/synchronizer.rs:97-143 maps these names).
FORM_HEADERS = ["타임스탬프", "이메일 주소", "이름", "소속", "SNUCSE ID (id.snucse.org 계정)", "사용할 서버",
                "GPU 개수", "vCPU 개수", "메모리 (GiB)", "스토리지 (GiB)", "MiG 개수", "요청 사유", "승인"]


def csv_escape(v):
    v = str(v)
    if any(c in v for c in ',"\n\r'):
        return '"' + v.replace('"', '""') + '"'
    return v


def make_csv(rows, headers=FORM_HEADERS):
    """rows: dicts with id_username, gpu_server, gpu, cpu, mem, storage, mig, authorized."""
    lines = [",".join(csv_escape(h) for h in headers)]
    for r in rows:
        vals = [r.get("timestamp", "2026/10/01 10:00:00"), r.get("email", f"{r['id_username']}@snu.ac.kr"),
                r.get("name", r["id_username"].upper()), r.get("department", "CSE"), r["id_username"],
                r.get("gpu_server", "mi355x-01"), r.get("gpu", 1), r.get("cpu", 8), r.get("mem", 64),
                r.get("storage", 100), r.get("mig", 0), r.get("description", "research"), r.get("authorized", "O")]
        lines.append(",".join(csv_escape(v) for v in vals))
    return "\r\n".join(lines) + "\r\n"


class FakeGoogle:
    def __init__(self, file_id="sheet-1", client_email="sync@bacchus.iam.gserviceaccount.com"):
        self.file_id = file_id
        self.client_email = client_email
        priv, pub = native().generate_rsa(2048)
        self.private_key, self.public_key = priv, pub
        self.csv = make_csv([])
        self.lock = threading.Lock()
        self.tokens = set()
        self.token_requests = 0
        self.export_requests = 0
        self.metadata_requests = 0
        self.version = 1
        self.rows = []
        self.fail_export = 0
        self.fail_token = 0
        self.export_delay = 0.0
        self.errors = []
        self.httpd = None
        self.thread = None

    # ---------------------------------------------------------------- setup
    def start(self):
        fg = self

        class Handler(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):  # quiet
                pass

            def _send(self, code, body, ctype="application/json"):
                data = body.encode() if isinstance(body, str) else body
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def do_POST(self):
                n = int(self.headers.get("Content-Length", "0"))
                body = self.rfile.read(n).decode()
                if self.path == "/_fake/rows":
                    req = json.loads(body or "{}")
                    fg.set_rows(req.get("rows", []), append=bool(req.get("append")))
                    return self._send(200, json.dumps({"version": fg.version}))
                if self.path != "/token":
                    return self._send(404, "{}")
                code, payload = fg._token(body)
                self._send(code, json.dumps(payload))

            def do_GET(self):
                code, payload, ctype = fg._export(self.path, self.headers.get("Authorization", ""))
                self._send(code, payload, ctype)

        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), Handler)
        self.httpd.daemon_threads = True
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)
        self.thread.start()
        return self

    def stop(self):
        if self.httpd:
            self.httpd.shutdown()
            self.httpd.server_close()

    @property
    def base(self):
        return f"http://127.0.0.1:{self.httpd.server_address[1]}"

    @property
    def token_url(self):
        return self.base + "/token"

    def service_account_json(self):
        return json.dumps({"type": "service_account", "project_id": "bacchus", "private_key_id": "kid-1",
                           "private_key": self.private_key, "client_email": self.client_email,
                           "client_id": "1", "token_uri": "https://oauth2.googleapis.com/token"})

    def env(self):
        """Test-only endpoint overrides for the synchronizer."""
        return {"BGC_GOOGLE_TOKEN_URL": self.token_url, "BGC_GOOGLE_API_BASE": self.base}

    def set_rows(self, rows, headers=FORM_HEADERS, append=False):
        with self.lock:
            self.rows = (self.rows + list(rows)) if append else list(rows)
            self.csv = make_csv(self.rows, headers)
            self.version += 1

    def set_csv(self, text):
        with self.lock:
            self.csv = text
            self.version += 1

    # ---------------------------------------------------------------- endpoints
    def _token(self, body):
        with self.lock:
            self.token_requests += 1
            if self.fail_token:
                return self.fail_token, {"error": "injected"}
        form = urllib.parse.parse_qs(body)
        if form.get("grant_type", [""])[0] != "urn:ietf:params:oauth:grant-type:jwt-bearer":
            return 400, {"error": "unsupported_grant_type"}
        jwt = form.get("assertion", [""])[0]
        try:
            head_b64, claims_b64, sig_b64 = jwt.split(".")
            n = native()
            sig = n.base64_decode(sig_b64)
            if not n.rs256_verify(self.public_key, head_b64 + "." + claims_b64, sig):
                return 400, {"error": "invalid_grant", "error_description": "bad signature"}
            header = json.loads(n.base64_decode(head_b64))
            claims = json.loads(n.base64_decode(claims_b64))
        except Exception as e:  # noqa: BLE001
            self.errors.append(str(e))
            return 400, {"error": "invalid_grant", "error_description": str(e)}
        now = time.time()
        problems = []
        if header.get("alg") != "RS256":
            problems.append("alg")
        if claims.get("iss") != self.client_email:
            problems.append("iss")
        if claims.get("aud") != "https://oauth2.googleapis.com/token":
            problems.append("aud")
        if claims.get("scope") != SCOPE:
            problems.append("scope")
        if not (claims.get("iat", 0) - 60 <= now <= claims.get("exp", 0)):
            problems.append("time")
        if problems:
            self.errors.append(f"claims: {problems}")
            return 400, {"error": "invalid_grant", "error_description": ",".join(problems)}
        tok = f"ya29.fake-{len(self.tokens)}"
        with self.lock:
            self.tokens.add(tok)
        return 200, {"access_token": tok, "expires_in": 3599, "token_type": "Bearer"}

    def _export(self, path, auth):
        u = urllib.parse.urlparse(path)
        q = urllib.parse.parse_qs(u.query)
        if u.path == f"/drive/v3/files/{self.file_id}":
            return self._metadata(q, auth)
        with self.lock:
            self.export_requests += 1
            fail = self.fail_export
            delay = self.export_delay
            csv = self.csv
            tokens = set(self.tokens)
        if delay:
            time.sleep(delay)
        if fail:
            return fail, json.dumps({"error": {"code": fail, "message": "injected"}}), "application/json"
        if not auth.startswith("Bearer ") or auth[7:] not in tokens:
            return 401, json.dumps({"error": {"code": 401, "message": "Invalid Credentials"}}), "application/json"
        if u.path != f"/drive/v3/files/{self.file_id}/export":
            return 404, json.dumps({"error": {"code": 404, "message": "File not found"}}), "application/json"
        if q.get("mimeType", [""])[0] != "text/csv":
            return 400, json.dumps({"error": {"code": 400, "message": "bad mimeType"}}), "application/json"
        return 200, csv.encode(), "text/csv"

    def _metadata(self, q, auth):
        with self.lock:
            self.metadata_requests += 1
            version = self.version
            tokens = set(self.tokens)
        if not auth.startswith("Bearer ") or auth[7:] not in tokens:
            return 401, json.dumps({"error": {"code": 401, "message": "Invalid Credentials"}}), "application/json"
        if q.get("fields", [""])[0] != "version":
            return 400, json.dumps({"error": {"code": 400, "message": "unsupported fields"}}), "application/json"
        return 200, json.dumps({"version": str(version)}), "application/json"
