"""P5: IAP / OIDC service-account request client -- the fork's delta (``auth.py``).

Behavioural reference: auth.py:17-38 (get_service_account_token), :40-44
(validate_credentials), :46-58 (get_signer_and_email), :60-76
(get_google_open_id_connect_token), :78-96 (make_request), :98-119 (main).

The flow is the reference's, implemented without google-auth (not shipped in this
image): find Application Default Credentials (``GOOGLE_APPLICATION_CREDENTIALS`` key
file, else the GCE metadata server), reject end-user credentials, build a signer (the
key's RSA key locally; on GCE the IAM Credentials ``signBlob`` API with the metadata
server's access token), mint a self-signed RS256 JWT whose ``target_audience`` is the IAP
OAuth client id, exchange it at ``oauth2/v4/token`` for a Google-signed ``id_token``,
then GET (or POST ``--input``) with ``Authorization: Bearer``.  Errors map as in the
reference: HTTP 403 -> PermissionError, connection failure -> ConnectionError, anything
else -> RuntimeError; missing credentials -> DefaultCredentialsError.

RSA (PKCS#1 v1.5 / SHA-256) signing and the PKCS#1 / PKCS#8 DER key parsing are done
with Python integers -- a one-shot signature per token, so speed is irrelevant.
"""
from __future__ import annotations

import base64
import hashlib
import json
import os
import time
import urllib.error
import urllib.parse
import urllib.request
from typing import Callable, Optional, Tuple

IAM_SCOPE = "https://www.googleapis.com/auth/iam"
OAUTH_TOKEN_URI = "https://www.googleapis.com/oauth2/v4/token"
JWT_GRANT_TYPE = "urn:ietf:params:oauth:grant-type:jwt-bearer"
METADATA = "http://metadata.google.internal/computeMetadata/v1"
SHA256_DIGEST_INFO = bytes.fromhex("3031300d060960864801650304020105000420")


class DefaultCredentialsError(Exception):
    pass


class RefreshError(Exception):
    pass


# (method, url, headers, body) -> (status, text); raises ConnectionError on network failure
Transport = Callable[[str, str, dict, Optional[bytes]], Tuple[int, str]]


def urllib_transport(method, url, headers, body):
    req = urllib.request.Request(url, data=body, method=method, headers=headers)
    try:
        with urllib.request.urlopen(req, timeout=30) as r:
            return r.status, r.read().decode()
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode(errors="replace")
    except (urllib.error.URLError, OSError) as e:
        raise ConnectionError(str(e))


# ------------------------------------------------------------------ DER / RSA
def _der_read(buf: bytes, i: int):
    tag = buf[i]
    ln = buf[i + 1]
    i += 2
    if ln & 0x80:
        n = ln & 0x7F
        ln = int.from_bytes(buf[i:i + n], "big")
        i += n
    return tag, buf[i:i + ln], i + ln


def _der_seq(buf: bytes):
    tag, body, _ = _der_read(buf, 0)
    if tag != 0x30:
        raise ValueError("expected DER SEQUENCE")
    out, i = [], 0
    while i < len(body):
        t, v, i = _der_read(body, i)
        out.append((t, v))
    return out


def parse_rsa_private_key(pem: str) -> Tuple[int, int, int]:
    """PKCS#1 ('RSA PRIVATE KEY') or PKCS#8 ('PRIVATE KEY') PEM -> (n, e, d)."""
    lines = [ln for ln in pem.strip().splitlines() if ln and not ln.startswith("-----")]
    der = base64.b64decode("".join(lines))
    items = _der_seq(der)
    if len(items) == 3 and items[2][0] == 0x04:        # PKCS#8: version, algId, OCTET STRING(PKCS#1)
        items = _der_seq(items[2][1])
    ints = [int.from_bytes(v, "big") for t, v in items if t == 0x02]
    # RSAPrivateKey: version, n, e, d, p, q, dp, dq, qinv
    return ints[1], ints[2], ints[3]


def rsa_sign_sha256(key: Tuple[int, int, int], msg: bytes) -> bytes:
    n, _, d = key
    k = (n.bit_length() + 7) // 8
    t = SHA256_DIGEST_INFO + hashlib.sha256(msg).digest()
    if k < len(t) + 11:
        raise ValueError("RSA key too short")
    em = b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t
    return pow(int.from_bytes(em, "big"), d, n).to_bytes(k, "big")


def rsa_verify_sha256(n: int, e: int, msg: bytes, sig: bytes) -> bool:
    k = (n.bit_length() + 7) // 8
    em = pow(int.from_bytes(sig, "big"), e, n).to_bytes(k, "big")
    t = SHA256_DIGEST_INFO + hashlib.sha256(msg).digest()
    return em == b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t


def b64url(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


# ------------------------------------------------------------------ credentials / signers
class KeySigner:
    def __init__(self, pem: str, key_id: Optional[str] = None):
        self.key = parse_rsa_private_key(pem)
        self.key_id = key_id

    def sign(self, msg: bytes) -> bytes:
        return rsa_sign_sha256(self.key, msg)


class IamSigner:
    """``google.auth.iam.Signer``: signBlob through the IAM Credentials API."""

    def __init__(self, transport: Transport, access_token: str, email: str):
        self.t, self.token, self.email = transport, access_token, email
        self.key_id = None

    def sign(self, msg: bytes) -> bytes:
        url = f"https://iamcredentials.googleapis.com/v1/projects/-/serviceAccounts/{self.email}:signBlob"
        code, text = self.t("POST", url, {"Authorization": f"Bearer {self.token}",
                                          "Content-Type": "application/json"},
                            json.dumps({"payload": base64.b64encode(msg).decode()}).encode())
        if code != 200:
            raise RefreshError(f"signBlob failed: HTTP {code} {text}")
        return base64.b64decode(json.loads(text)["signedBlob"])


class Credentials:
    kind = "service_account"

    def __init__(self, email: str, signer, compute_engine: bool = False):
        self.service_account_email = email
        self.signer = signer
        self.compute_engine = compute_engine


class UserCredentials:
    kind = "authorized_user"


def default_credentials(transport: Transport = urllib_transport, env=None):
    """ADC discovery (key file, then GCE metadata)."""
    env = os.environ if env is None else env
    path = env.get("GOOGLE_APPLICATION_CREDENTIALS")
    if path:
        try:
            with open(path) as f:
                info = json.load(f)
        except (OSError, ValueError) as e:
            raise DefaultCredentialsError(f"File {path} could not be loaded: {e}")
        if info.get("type") == "authorized_user":
            return UserCredentials()
        if info.get("type") != "service_account":
            raise DefaultCredentialsError(f"unsupported credentials type {info.get('type')!r}")
        return Credentials(info["client_email"], KeySigner(info["private_key"], info.get("private_key_id")))
    try:
        code, email = transport("GET", f"{METADATA}/instance/service-accounts/default/email",
                                {"Metadata-Flavor": "Google"}, None)
    except ConnectionError:
        code = 0
    if code != 200:
        raise DefaultCredentialsError("Could not automatically determine credentials.")
    code, tok = transport("GET", f"{METADATA}/instance/service-accounts/default/token?"
                          + urllib.parse.urlencode({"scopes": IAM_SCOPE}), {"Metadata-Flavor": "Google"}, None)
    if code != 200:
        raise RefreshError(f"metadata token refresh failed: HTTP {code}")
    return Credentials(email.strip(), IamSigner(transport, json.loads(tok)["access_token"], email.strip()),
                       compute_engine=True)


def validate_credentials(creds):
    if isinstance(creds, UserCredentials):
        raise TypeError("This script is only supported for service accounts.")


def get_signer_and_email(creds):
    return creds.service_account_email, creds.signer


def make_assertion(signer, email: str, client_id: str, now: Optional[float] = None) -> str:
    now = int(now if now is not None else time.time())
    header = {"alg": "RS256", "typ": "JWT"}
    if getattr(signer, "key_id", None):
        header["kid"] = signer.key_id
    claims = {"iss": email, "sub": email, "aud": OAUTH_TOKEN_URI, "iat": now, "exp": now + 3600,
              "target_audience": client_id}
    signing_input = (b64url(json.dumps(header, separators=(",", ":")).encode()) + "." +
                     b64url(json.dumps(claims, separators=(",", ":")).encode())).encode()
    return signing_input.decode() + "." + b64url(signer.sign(signing_input))


def get_google_open_id_connect_token(signer, email, client_id, transport: Transport = urllib_transport) -> str:
    try:
        body = urllib.parse.urlencode({"assertion": make_assertion(signer, email, client_id),
                                       "grant_type": JWT_GRANT_TYPE}).encode()
        code, text = transport("POST", OAUTH_TOKEN_URI, {"Content-Type": "application/x-www-form-urlencoded"}, body)
        if code != 200:
            raise RuntimeError(f"token endpoint HTTP {code}: {text}")
        return json.loads(text)["id_token"]
    except Exception as e:
        raise RuntimeError(f"Failed to obtain OpenID Connect token: {e}")


def get_service_account_token(client_id: str, transport: Transport = urllib_transport, env=None):
    try:
        creds = default_credentials(transport, env)
    except DefaultCredentialsError as e:
        raise DefaultCredentialsError(f"Failed to obtain default credentials: {e}")
    validate_credentials(creds)
    email, signer = get_signer_and_email(creds)
    return get_google_open_id_connect_token(signer, email, client_id, transport), email


def make_request(url: str, token: str, data: Optional[str] = None, transport: Transport = urllib_transport) -> str:
    headers = {"Authorization": f"Bearer {token}"}
    try:
        code, text = transport("POST" if data else "GET", url, headers, data.encode() if data else None)
    except ConnectionError as e:
        raise ConnectionError(f"Failed to connect to the application: {e}")
    if code == 403:
        raise PermissionError("Service account does not have permission to access the IAP-protected application.")
    if code >= 400:
        raise RuntimeError(f"Bad response from application: {code} {text}")
    return text


def main(argv=None, transport: Transport = urllib_transport) -> int:
    import argparse
    p = argparse.ArgumentParser()
    p.add_argument("url", help="URL of the host model")
    p.add_argument("client_id", help="The client id used to setup IAP")
    p.add_argument("--input", help="The input file.")
    a = p.parse_args(argv)
    try:
        token, _ = get_service_account_token(a.client_id, transport)
        data = open(a.input).read() if a.input else None
        print(make_request(a.url, token, data, transport))
        return 0
    except (DefaultCredentialsError, PermissionError, ConnectionError, RuntimeError, TypeError) as e:
        print(f"Error: {e}")
        return 1
