"""Cloud IAM backends for the Profile controller plugins (G2a / G2b), over plain HTTPS.

Reference: components/profile-controller/controllers/plugin_workload_identity.go:90-132
(GCP IAM ``projects.serviceAccounts.getIamPolicy`` / ``setIamPolicy`` with Application Default
Credentials; the workload-identity member uses the credentials' project id when it has one)
and plugin_iam.go:75-126 (AWS IAM ``GetRole`` -> URL-decoded ``AssumeRolePolicyDocument`` ->
``UpdateAssumeRolePolicy``).  The reference links the Google and AWS SDKs; neither exists on
this platform, so both protocols are spoken directly:

* GCP: an OAuth2 access token for ``cloud-platform`` from the GCE/GKE metadata server or from
  a service-account key file (RS256 JWT-bearer grant, signed by ``utils.iap``'s RSA code),
  cached until shortly before expiry; JSON REST calls to ``iam.googleapis.com/v1``.
* AWS: credentials from the environment, from an IRSA web-identity token (STS
  ``AssumeRoleWithWebIdentity``, which needs no signature) or from the shared credentials
  file; IAM Query API calls (``Version=2010-05-08``) signed with Signature Version 4.

Every network call goes through a ``transport(method, url, headers, body) -> (status, text)``
callable (``utils.iap.urllib_transport`` by default), which the tests replace with recorded
request/response fixtures.
"""
from __future__ import annotations

import configparser
import datetime as _dt
import hashlib
import hmac
import json
import os
import threading
import time
import urllib.parse
import xml.etree.ElementTree as ET
from typing import Callable, Dict, Optional, Tuple

from ..utils import iap
from .profile import IamBackend, InMemoryIam

Transport = Callable[[str, str, dict, Optional[bytes]], Tuple[int, str]]

CLOUD_PLATFORM_SCOPE = "https://www.googleapis.com/auth/cloud-platform"
GCP_IAM_ENDPOINT = "https://iam.googleapis.com/v1"
AWS_IAM_ENDPOINT = "https://iam.amazonaws.com/"
AWS_IAM_VERSION = "2010-05-08"
AWS_IAM_NS = "{https://iam.amazonaws.com/doc/2010-05-08/}"
AWS_STS_NS = "{https://sts.amazonaws.com/doc/2011-06-15/}"


class CloudIamError(RuntimeError):
    pass


# ============================================================================ GCP
class GcpToken:
    """Cached OAuth2 access token (ADC: key file, else the metadata server)."""

    def __init__(self, transport: Transport = iap.urllib_transport, env=None, scope: str = CLOUD_PLATFORM_SCOPE,
                 clock: Callable[[], float] = time.time):
        self.t, self.env, self.scope, self.clock = transport, (os.environ if env is None else env), scope, clock
        self._tok: Optional[str] = None
        self._exp = 0.0
        self._project: Optional[str] = None
        self._lock = threading.Lock()

    def _key_file(self) -> Optional[dict]:
        path = self.env.get("GOOGLE_APPLICATION_CREDENTIALS")
        if not path:
            return None
        try:
            with open(path) as f:
                info = json.load(f)
        except (OSError, ValueError) as e:
            raise iap.DefaultCredentialsError(f"File {path} could not be loaded: {e}")
        if info.get("type") != "service_account":
            raise iap.DefaultCredentialsError(f"unsupported credentials type {info.get('type')!r}")
        return info

    def _refresh(self) -> Tuple[str, float]:
        info = self._key_file()
        now = self.clock()
        if info is not None:
            signer = iap.KeySigner(info["private_key"], info.get("private_key_id"))
            header = {"alg": "RS256", "typ": "JWT"}
            if signer.key_id:
                header["kid"] = signer.key_id
            claims = {"iss": info["client_email"], "scope": self.scope, "aud": info.get("token_uri", iap.OAUTH_TOKEN_URI),
                      "iat": int(now), "exp": int(now) + 3600}
            signing_input = (iap.b64url(json.dumps(header, separators=(",", ":")).encode()) + "." +
                             iap.b64url(json.dumps(claims, separators=(",", ":")).encode()))
            assertion = signing_input + "." + iap.b64url(signer.sign(signing_input.encode()))
            body = urllib.parse.urlencode({"grant_type": iap.JWT_GRANT_TYPE, "assertion": assertion}).encode()
            code, text = self.t("POST", claims["aud"], {"Content-Type": "application/x-www-form-urlencoded"}, body)
        else:
            url = f"{iap.METADATA}/instance/service-accounts/default/token?" + urllib.parse.urlencode(
                {"scopes": self.scope})
            code, text = self.t("GET", url, {"Metadata-Flavor": "Google"}, None)
        if code != 200:
            raise iap.RefreshError(f"GCP token refresh failed: HTTP {code} {text[:200]}")
        d = json.loads(text)
        return d["access_token"], now + float(d.get("expires_in", 3600))

    def token(self) -> str:
        with self._lock:
            if self._tok is None or self.clock() > self._exp - 60:
                self._tok, self._exp = self._refresh()
            return self._tok

    def project_id(self) -> str:
        """The credentials' project (key file ``project_id``, metadata ``project/project-id`` or
        ``GOOGLE_CLOUD_PROJECT``); "" when none is known."""
        if self._project is None:
            proj = self.env.get("GOOGLE_CLOUD_PROJECT", "")
            info = self._key_file()
            if info is not None:
                proj = info.get("project_id", proj)
            elif not proj:
                try:
                    code, text = self.t("GET", f"{iap.METADATA}/project/project-id", {"Metadata-Flavor": "Google"}, None)
                    proj = text.strip() if code == 200 else ""
                except ConnectionError:
                    proj = ""
            self._project = proj
        return self._project


class GcpIam(IamBackend):
    """``projects.serviceAccounts.getIamPolicy`` / ``setIamPolicy`` over the IAM REST API."""

    def __init__(self, transport: Transport = iap.urllib_transport, env=None, token: Optional[GcpToken] = None):
        self.t = transport
        self.tok = token or GcpToken(transport, env)

    def _call(self, resource: str, method: str, body: dict) -> dict:
        url = f"{GCP_IAM_ENDPOINT}/{resource}:{method}"
        code, text = self.t("POST", url, {"Authorization": f"Bearer {self.tok.token()}",
                                          "Content-Type": "application/json"}, json.dumps(body).encode())
        if code != 200:
            raise CloudIamError(f"GCP IAM {method} {resource}: HTTP {code} {text[:300]}")
        return json.loads(text or "{}")

    def gcp_get_policy(self, resource: str) -> dict:
        pol = self._call(resource, "getIamPolicy", {})
        pol.setdefault("bindings", [])
        return pol

    def gcp_set_policy(self, resource: str, policy: dict):
        # the policy carries the etag read by getIamPolicy: a concurrent writer makes this fail
        # (HTTP 409) instead of being overwritten, and the reconcile is retried
        self._call(resource, "setIamPolicy", {"policy": policy})

    def gcp_default_project(self) -> str:
        return self.tok.project_id()


# ============================================================================ AWS
def _hmac(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode(), hashlib.sha256).digest()


def sigv4_sign(method: str, url: str, headers: Dict[str, str], body: bytes, access_key: str, secret_key: str,
               region: str, service: str, amz_date: str, session_token: Optional[str] = None) -> Dict[str, str]:
    """AWS Signature Version 4 (header form).  Returns ``headers`` plus ``X-Amz-Date``,
    ``X-Amz-Security-Token`` (temporary credentials) and ``Authorization``."""
    u = urllib.parse.urlsplit(url)
    out = dict(headers)
    out["X-Amz-Date"] = amz_date
    if session_token:
        out["X-Amz-Security-Token"] = session_token
    host = u.netloc
    canon = {"host": host}
    for k, v in out.items():
        canon[k.lower().strip()] = " ".join(str(v).strip().split())
    signed = ";".join(sorted(canon))
    canon_headers = "".join(f"{k}:{canon[k]}\n" for k in sorted(canon))
    q = urllib.parse.parse_qsl(u.query, keep_blank_values=True)
    canon_query = "&".join(f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(v, safe='-_.~')}"
                           for k, v in sorted(q))
    path = urllib.parse.quote(u.path or "/", safe="/-_.~")
    payload_hash = hashlib.sha256(body or b"").hexdigest()
    creq = "\n".join([method.upper(), path, canon_query, canon_headers, signed, payload_hash])
    date = amz_date[:8]
    scope = f"{date}/{region}/{service}/aws4_request"
    sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(creq.encode()).hexdigest()])
    k = _hmac(_hmac(_hmac(_hmac(("AWS4" + secret_key).encode(), date), region), service), "aws4_request")
    sig = hmac.new(k, sts.encode(), hashlib.sha256).hexdigest()
    out["Authorization"] = (f"AWS4-HMAC-SHA256 Credential={access_key}/{scope}, SignedHeaders={signed}, "
                            f"Signature={sig}")
    return out


class AwsCredentials:
    """Credential chain: environment -> IRSA web identity (STS) -> shared credentials file."""

    def __init__(self, transport: Transport = iap.urllib_transport, env=None, clock: Callable[[], float] = time.time):
        self.t, self.env, self.clock = transport, (os.environ if env is None else env), clock
        self._cached: Optional[Tuple[str, str, Optional[str], float]] = None
        self._lock = threading.Lock()

    def _web_identity(self) -> Optional[Tuple[str, str, str, float]]:
        role, tok_file = self.env.get("AWS_ROLE_ARN"), self.env.get("AWS_WEB_IDENTITY_TOKEN_FILE")
        if not (role and tok_file):
            return None
        with open(tok_file) as f:
            token = f.read().strip()
        region = self.env.get("AWS_REGION") or self.env.get("AWS_DEFAULT_REGION")
        host = f"https://sts.{region}.amazonaws.com/" if region else "https://sts.amazonaws.com/"
        body = urllib.parse.urlencode({"Action": "AssumeRoleWithWebIdentity", "Version": "2011-06-15",
                                       "RoleArn": role, "RoleSessionName": self.env.get("AWS_ROLE_SESSION_NAME",
                                                                                        "kfamd-profile-controller"),
                                       "WebIdentityToken": token}).encode()
        code, text = self.t("POST", host, {"Content-Type": "application/x-www-form-urlencoded"}, body)
        if code != 200:
            raise CloudIamError(f"STS AssumeRoleWithWebIdentity: HTTP {code} {text[:300]}")
        c = ET.fromstring(text).find(f"{AWS_STS_NS}AssumeRoleWithWebIdentityResult/{AWS_STS_NS}Credentials")
        exp = _dt.datetime.strptime(c.findtext(f"{AWS_STS_NS}Expiration")[:19], "%Y-%m-%dT%H:%M:%S").replace(
            tzinfo=_dt.timezone.utc).timestamp()
        return (c.findtext(f"{AWS_STS_NS}AccessKeyId"), c.findtext(f"{AWS_STS_NS}SecretAccessKey"),
                c.findtext(f"{AWS_STS_NS}SessionToken"), exp)

    def get(self) -> Tuple[str, str, Optional[str]]:
        with self._lock:
            if self._cached and self.clock() < self._cached[3] - 300:
                return self._cached[:3]
            e = self.env
            if e.get("AWS_ACCESS_KEY_ID") and e.get("AWS_SECRET_ACCESS_KEY"):
                self._cached = (e["AWS_ACCESS_KEY_ID"], e["AWS_SECRET_ACCESS_KEY"], e.get("AWS_SESSION_TOKEN"),
                                float("inf"))
                return self._cached[:3]
            wi = self._web_identity()
            if wi is not None:
                self._cached = wi
                return wi[:3]
            path = e.get("AWS_SHARED_CREDENTIALS_FILE") or os.path.expanduser("~/.aws/credentials")
            cp = configparser.ConfigParser()
            if cp.read(path):
                sec = cp[e.get("AWS_PROFILE", "default")]
                self._cached = (sec["aws_access_key_id"], sec["aws_secret_access_key"],
                                sec.get("aws_session_token"), float("inf"))
                return self._cached[:3]
            raise CloudIamError("no AWS credentials (env, web identity token or shared credentials file)")


class AwsIam(IamBackend):
    """IAM ``GetRole`` / ``UpdateAssumeRolePolicy`` (Query API, SigV4, global endpoint us-east-1)."""

    def __init__(self, transport: Transport = iap.urllib_transport, env=None, creds: Optional[AwsCredentials] = None,
                 clock: Callable[[], float] = time.time):
        self.t, self.clock = transport, clock
        self.creds = creds or AwsCredentials(transport, env, clock)

    def _call(self, params: dict) -> ET.Element:
        body = urllib.parse.urlencode(dict(params, Version=AWS_IAM_VERSION)).encode()
        ak, sk, st = self.creds.get()
        amz_date = _dt.datetime.fromtimestamp(self.clock(), _dt.timezone.utc).strftime("%Y%m%dT%H%M%SZ")
        headers = sigv4_sign("POST", AWS_IAM_ENDPOINT,
                             {"Content-Type": "application/x-www-form-urlencoded; charset=utf-8"}, body,
                             ak, sk, "us-east-1", "iam", amz_date, st)
        code, text = self.t("POST", AWS_IAM_ENDPOINT, headers, body)
        if code != 200:
            raise CloudIamError(f"AWS IAM {params.get('Action')}: HTTP {code} {text[:300]}")
        return ET.fromstring(text)

    def aws_get_assume_role_policy(self, role_name: str) -> str:
        root = self._call({"Action": "GetRole", "RoleName": role_name})
        doc = root.findtext(f"{AWS_IAM_NS}GetRoleResult/{AWS_IAM_NS}Role/{AWS_IAM_NS}AssumeRolePolicyDocument")
        if doc is None:
            raise CloudIamError(f"GetRole {role_name}: no AssumeRolePolicyDocument in the response")
        return urllib.parse.unquote(doc)          # the document is URL-encoded (plugin_iam.go:103)

    def aws_update_assume_role_policy(self, role_name: str, doc: str):
        self._call({"Action": "UpdateAssumeRolePolicy", "RoleName": role_name, "PolicyDocument": doc})


# ============================================================================ selection
class CloudIam(IamBackend):
    """The controller's default backend: GCP calls go to :class:`GcpIam`, AWS calls to
    :class:`AwsIam`, each created on first use (a cluster that configures only one of the
    plugins never needs the other cloud's credentials)."""

    def __init__(self, transport: Transport = iap.urllib_transport, env=None):
        self.t, self.env = transport, env
        self._gcp: Optional[GcpIam] = None
        self._aws: Optional[AwsIam] = None

    @property
    def gcp(self) -> GcpIam:
        if self._gcp is None:
            self._gcp = GcpIam(self.t, self.env)
        return self._gcp

    @property
    def aws(self) -> AwsIam:
        if self._aws is None:
            self._aws = AwsIam(self.t, self.env)
        return self._aws

    def gcp_get_policy(self, resource):
        return self.gcp.gcp_get_policy(resource)

    def gcp_set_policy(self, resource, policy):
        self.gcp.gcp_set_policy(resource, policy)

    def gcp_default_project(self):
        return self.gcp.gcp_default_project()

    def aws_get_assume_role_policy(self, role_name):
        return self.aws.aws_get_assume_role_policy(role_name)

    def aws_update_assume_role_policy(self, role_name, doc):
        self.aws.aws_update_assume_role_policy(role_name, doc)


def iam_backend(kind: Optional[str] = None) -> IamBackend:
    """``KFAMD_IAM_BACKEND=cloud`` (default for the deployed controller) or ``memory`` (local
    cluster / tests: the in-process model of both clouds)."""
    kind = kind or os.environ.get("KFAMD_IAM_BACKEND", "cloud")
    return InMemoryIam() if kind == "memory" else CloudIam()
