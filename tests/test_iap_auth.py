"""IAP client (fork delta auth.py) with a fake Google token endpoint / IAP app.
Parity: the reference's flow (auth.py:17-119); google-auth is not installed here, so the
exchange is checked against a fake transport and a locally generated RSA key."""
import base64
import json
import shutil
import subprocess

import pytest

from service_account_auth_improvements_amd.utils import iap


def _b64d(s):
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


@pytest.fixture
def keyfile(tmp_path):
    if shutil.which("openssl") is None:
        pytest.skip("openssl not available")
    pem = subprocess.run(["openssl", "genpkey", "-algorithm", "RSA", "-pkeyopt", "rsa_keygen_bits:2048"],
                         capture_output=True, text=True, check=True).stdout
    f = tmp_path / "sa.json"
    f.write_text(json.dumps({"type": "service_account", "client_email": "ci@proj.iam.gserviceaccount.com",
                             "private_key": pem, "private_key_id": "k1"}))
    return f, pem


class FakeGoogle:
    def __init__(self, key, app_status=200):
        self.n, self.e, _ = key
        self.app_status = app_status
        self.calls = []

    def __call__(self, method, url, headers, body):
        self.calls.append((method, url, headers, body))
        if url == iap.OAUTH_TOKEN_URI:
            form = dict(x.split("=", 1) for x in body.decode().split("&"))
            assert form["grant_type"] == "urn%3Aietf%3Aparams%3Aoauth%3Agrant-type%3Ajwt-bearer"
            h, c, s = form["assertion"].split(".")
            assert iap.rsa_verify_sha256(self.n, self.e, f"{h}.{c}".encode(), _b64d(s))
            claims = json.loads(_b64d(c))
            assert claims["target_audience"] == "client-123.apps.googleusercontent.com"
            assert json.loads(_b64d(h))["kid"] == "k1"
            return 200, json.dumps({"id_token": "ID." + claims["iss"]})
        assert headers["Authorization"] == "Bearer ID.ci@proj.iam.gserviceaccount.com"
        return self.app_status, "hello from IAP app" if self.app_status == 200 else "denied"


def test_token_and_request(keyfile, capsys):
    f, pem = keyfile
    fake = FakeGoogle(iap.parse_rsa_private_key(pem))
    tok, email = iap.get_service_account_token("client-123.apps.googleusercontent.com", fake,
                                               env={"GOOGLE_APPLICATION_CREDENTIALS": str(f)})
    assert email == "ci@proj.iam.gserviceaccount.com" and tok == "ID." + email
    assert iap.make_request("https://app.example.com/", tok, None, fake) == "hello from IAP app"
    assert fake.calls[-1][0] == "GET"
    assert iap.make_request("https://app.example.com/", tok, '{"x":1}', fake) == "hello from IAP app"
    assert fake.calls[-1][0] == "POST" and fake.calls[-1][3] == b'{"x":1}'


def test_error_mapping(keyfile, monkeypatch):
    f, pem = keyfile
    fake = FakeGoogle(iap.parse_rsa_private_key(pem), app_status=403)
    with pytest.raises(PermissionError):
        iap.make_request("https://app.example.com/", "ID.ci@proj.iam.gserviceaccount.com", None, fake)
    fake.app_status = 500
    with pytest.raises(RuntimeError):
        iap.make_request("https://app.example.com/", "ID.ci@proj.iam.gserviceaccount.com", None, fake)

    def down(*a):
        raise ConnectionError("refused")
    with pytest.raises(ConnectionError):
        iap.make_request("https://app.example.com/", "t", None, down)
    with pytest.raises(iap.DefaultCredentialsError):
        iap.get_service_account_token("c", down, env={})


def test_user_credentials_rejected(tmp_path):
    f = tmp_path / "user.json"
    f.write_text(json.dumps({"type": "authorized_user", "client_id": "x", "refresh_token": "y"}))
    with pytest.raises(TypeError, match="only supported for service accounts"):
        iap.get_service_account_token("c", lambda *a: (500, ""), env={"GOOGLE_APPLICATION_CREDENTIALS": str(f)})


def test_gce_metadata_signer():
    signed = []

    def t(method, url, headers, body):
        if url.endswith("/default/email"):
            return 200, "vm@proj.iam.gserviceaccount.com"
        if "/default/token" in url:
            return 200, json.dumps({"access_token": "AT"})
        if ":signBlob" in url:
            assert headers["Authorization"] == "Bearer AT"
            signed.append(body)
            return 200, json.dumps({"signedBlob": base64.b64encode(b"sig").decode()})
        if url == iap.OAUTH_TOKEN_URI:
            return 200, json.dumps({"id_token": "GCE-ID"})
        raise AssertionError(url)
    tok, email = iap.get_service_account_token("cid", t, env={})
    assert tok == "GCE-ID" and email == "vm@proj.iam.gserviceaccount.com" and len(signed) == 1


def test_cli_main(keyfile, tmp_path, capsys, monkeypatch):
    f, pem = keyfile
    monkeypatch.setenv("GOOGLE_APPLICATION_CREDENTIALS", str(f))
    fake = FakeGoogle(iap.parse_rsa_private_key(pem))
    inp = tmp_path / "in.json"
    inp.write_text('{"instances": [1]}')
    assert iap.main(["https://app/", "client-123.apps.googleusercontent.com", "--input", str(inp)], fake) == 0
    assert "hello from IAP app" in capsys.readouterr().out
    fake.app_status = 403
    assert iap.main(["https://app/", "client-123.apps.googleusercontent.com"], fake) == 1
    assert "Error: Service account does not have permission" in capsys.readouterr().out
