"""Cloud IAM backends of the Profile plugins at the transport layer:
SigV4 against published AWS signing examples, and recorded request/response fixtures for the
GCP IAM REST calls (metadata-server and key-file tokens) and the AWS IAM Query calls (env and
IRSA web-identity credentials), end to end through the Profile controller.
Reference: profile-controller/controllers/plugin_workload_identity.go:90-160, plugin_iam.go:75-255."""
import json
import shutil
import subprocess
import urllib.parse

import pytest

from service_account_auth_improvements_amd.controlplane import cloud_iam
from service_account_auth_improvements_amd.controlplane.cloud_iam import (AwsCredentials, AwsIam, CloudIam, GcpIam,
                                                                          GcpToken, sigv4_sign)
from service_account_auth_improvements_amd.utils import iap

T0 = 1440938160.0     # 2015-08-30T12:36:00Z, the date of the AWS SigV4 examples


# ------------------------------------------------------------------ SigV4
def test_sigv4_get_vanilla_example():
    """aws-sig-v4-test-suite 'get-vanilla'."""
    h = sigv4_sign("GET", "https://example.amazonaws.com/", {}, b"", "AKIDEXAMPLE",
                   "wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY", "us-east-1", "service", "20150830T123600Z")
    assert h["Authorization"] == ("AWS4-HMAC-SHA256 Credential=AKIDEXAMPLE/20150830/us-east-1/service/aws4_request, "
                                  "SignedHeaders=host;x-amz-date, "
                                  "Signature=5fa00fa31553b73ebf1942676e86291e8372ff2a2260956d9b8aae1d763fbf31")


def test_sigv4_iam_list_users_example():
    """The IAM example of the AWS SigV4 documentation (GET ?Action=ListUsers&Version=2010-05-08)."""
    h = sigv4_sign("GET", "https://iam.amazonaws.com/?Action=ListUsers&Version=2010-05-08",
                   {"Content-Type": "application/x-www-form-urlencoded; charset=utf-8"}, b"", "AKIDEXAMPLE",
                   "wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY", "us-east-1", "iam", "20150830T123600Z")
    assert h["Authorization"].endswith("SignedHeaders=content-type;host;x-amz-date, "
                                       "Signature=5d672d79c15b13162d9279b0855cfba6789a8edb4c82c400e06b5924a6f2b5d7")


# ------------------------------------------------------------------ fixtures
class Recorder:
    def __init__(self, routes):
        self.routes, self.calls = routes, []

    def __call__(self, method, url, headers, body):
        self.calls.append({"method": method, "url": url, "headers": dict(headers), "body": body})
        for match, resp in self.routes:
            if match(method, url, headers, body):
                return resp(method, url, headers, body) if callable(resp) else resp
        raise AssertionError(f"unexpected request {method} {url}")


SA_RES = "projects/gcp-proj/serviceAccounts/kf-user@gcp-proj.iam.gserviceaccount.com"


def _gcp_routes(policy_store, token="ya29.meta"):
    def get_pol(m, u, h, b):
        assert h["Authorization"] == f"Bearer {token}" and json.loads(b) == {}
        return 200, json.dumps(policy_store["p"])

    def set_pol(m, u, h, b):
        assert h["Authorization"] == f"Bearer {token}" and h["Content-Type"] == "application/json"
        policy_store["p"] = json.loads(b)["policy"]
        return 200, json.dumps(policy_store["p"])
    return [
        (lambda m, u, h, b: u.startswith(iap.METADATA + "/instance/service-accounts/default/token"),
         (200, json.dumps({"access_token": token, "expires_in": 3599, "token_type": "Bearer"}))),
        (lambda m, u, h, b: u == iap.METADATA + "/project/project-id", (200, "cluster-proj")),
        (lambda m, u, h, b: u == f"https://iam.googleapis.com/v1/{SA_RES}:getIamPolicy", get_pol),
        (lambda m, u, h, b: u == f"https://iam.googleapis.com/v1/{SA_RES}:setIamPolicy", set_pol),
    ]


def test_gcp_metadata_token_policy_round_trip():
    store = {"p": {"etag": "BwX1", "bindings": [{"role": "roles/viewer", "members": ["user:a@x.com"]}]}}
    rec = Recorder(_gcp_routes(store))
    g = GcpIam(rec, env={})
    pol = g.gcp_get_policy(SA_RES)
    pol["bindings"].append({"role": "roles/iam.workloadIdentityUser", "members": ["serviceAccount:m"]})
    g.gcp_set_policy(SA_RES, pol)
    assert g.gcp_default_project() == "cluster-proj"
    urls = [c["url"] for c in rec.calls]
    assert sum("service-accounts/default/token" in u for u in urls) == 1, "token is cached"
    tok = next(c for c in rec.calls if "default/token" in c["url"])
    assert tok["headers"] == {"Metadata-Flavor": "Google"}
    assert urllib.parse.parse_qs(urllib.parse.urlsplit(tok["url"]).query)["scopes"] == [cloud_iam.CLOUD_PLATFORM_SCOPE]
    assert store["p"]["etag"] == "BwX1" and len(store["p"]["bindings"]) == 2   # etag sent back: no blind overwrite


def test_gcp_http_error_is_raised():
    rec = Recorder([(lambda m, u, h, b: "default/token" in u, (200, json.dumps({"access_token": "t"}))),
                    (lambda m, u, h, b: u.endswith(":getIamPolicy"), (403, '{"error": {"status": "PERMISSION_DENIED"}}'))])
    with pytest.raises(cloud_iam.CloudIamError, match="HTTP 403"):
        GcpIam(rec, env={}).gcp_get_policy(SA_RES)


@pytest.fixture
def keyfile(tmp_path):
    if shutil.which("openssl") is None:
        pytest.skip("openssl not available")
    pem = subprocess.run(["openssl", "genpkey", "-algorithm", "RSA", "-pkeyopt", "rsa_keygen_bits:2048"],
                         capture_output=True, text=True, check=True).stdout
    f = tmp_path / "sa.json"
    f.write_text(json.dumps({"type": "service_account", "client_email": "ctl@key-proj.iam.gserviceaccount.com",
                             "private_key": pem, "private_key_id": "k9", "project_id": "key-proj",
                             "token_uri": "https://oauth2.googleapis.com/token"}))
    return str(f), iap.parse_rsa_private_key(pem)


def test_gcp_key_file_jwt_bearer_grant(keyfile):
    path, (n, e, _) = keyfile

    def token(m, u, h, b):
        form = dict(urllib.parse.parse_qsl(b.decode()))
        assert form["grant_type"] == iap.JWT_GRANT_TYPE
        hd, cl, sg = form["assertion"].split(".")
        dec = lambda s: __import__("base64").urlsafe_b64decode(s + "=" * (-len(s) % 4))   # noqa: E731
        assert iap.rsa_verify_sha256(n, e, f"{hd}.{cl}".encode(), dec(sg))
        claims = json.loads(dec(cl))
        assert claims["scope"] == cloud_iam.CLOUD_PLATFORM_SCOPE and claims["aud"] == u
        assert claims["iss"] == "ctl@key-proj.iam.gserviceaccount.com" and json.loads(dec(hd))["kid"] == "k9"
        return 200, json.dumps({"access_token": "ya29.key", "expires_in": 3600})
    store = {"p": {"bindings": []}}
    routes = [(lambda m, u, h, b: u == "https://oauth2.googleapis.com/token", token)] + _gcp_routes(store, "ya29.key")[2:]
    rec = Recorder(routes)
    g = GcpIam(rec, env={"GOOGLE_APPLICATION_CREDENTIALS": path})
    assert g.gcp_get_policy(SA_RES) == {"bindings": []}
    assert g.gcp_default_project() == "key-proj"


# ------------------------------------------------------------------ AWS
ROLE_DOC = {"Version": "2012-10-17", "Statement": [{
    "Effect": "Allow", "Action": "sts:AssumeRoleWithWebIdentity",
    "Principal": {"Federated": "arn:aws:iam::123456789012:oidc-provider/oidc.eks.us-west-2.amazonaws.com/id/ABC"},
    "Condition": {"StringEquals": {"oidc.eks.us-west-2.amazonaws.com/id/ABC:aud": ["sts.amazonaws.com"]}}}]}


def _get_role_xml(doc):
    return ('<GetRoleResponse xmlns="https://iam.amazonaws.com/doc/2010-05-08/"><GetRoleResult><Role>'
            f'<RoleName>kf-user</RoleName><AssumeRolePolicyDocument>{urllib.parse.quote(json.dumps(doc))}'
            '</AssumeRolePolicyDocument></Role></GetRoleResult></GetRoleResponse>')


def _aws_routes(state):
    def iam(m, u, h, b):
        form = dict(urllib.parse.parse_qsl(b.decode()))
        assert form["Version"] == "2010-05-08"
        # the signature must verify: re-sign the same request and compare
        again = sigv4_sign("POST", u, {"Content-Type": h["Content-Type"]}, b, state["ak"], state["sk"], "us-east-1",
                           "iam", h["X-Amz-Date"], h.get("X-Amz-Security-Token"))
        assert h["Authorization"] == again["Authorization"]
        assert h["Authorization"].startswith(f"AWS4-HMAC-SHA256 Credential={state['ak']}/20150830/us-east-1/iam/")
        if form["Action"] == "GetRole":
            assert form["RoleName"] == "kf-user"
            return 200, _get_role_xml(state["doc"])
        assert form["Action"] == "UpdateAssumeRolePolicy" and form["RoleName"] == "kf-user"
        state["doc"] = json.loads(form["PolicyDocument"])
        return 200, '<UpdateAssumeRolePolicyResponse xmlns="https://iam.amazonaws.com/doc/2010-05-08/"/>'
    return [(lambda m, u, h, b: u == "https://iam.amazonaws.com/" and m == "POST", iam)]


def test_aws_env_credentials_get_and_update_role():
    state = {"doc": ROLE_DOC, "ak": "AKIDENV", "sk": "secretenv"}
    rec = Recorder(_aws_routes(state))
    a = AwsIam(rec, env={"AWS_ACCESS_KEY_ID": "AKIDENV", "AWS_SECRET_ACCESS_KEY": "secretenv"}, clock=lambda: T0)
    doc = a.aws_get_assume_role_policy("kf-user")
    assert json.loads(doc) == ROLE_DOC                       # URL-decoded
    a.aws_update_assume_role_policy("kf-user", json.dumps({"x": 1}))
    assert state["doc"] == {"x": 1}
    assert all("X-Amz-Date" in c["headers"] and c["headers"]["X-Amz-Date"] == "20150830T123600Z" for c in rec.calls)


def test_aws_irsa_web_identity_credentials(tmp_path):
    tok = tmp_path / "token"
    tok.write_text("eyJhbGciOi.web.identity\n")
    state = {"doc": ROLE_DOC, "ak": "ASIATEMP", "sk": "tempsecret"}

    def sts(m, u, h, b):
        form = dict(urllib.parse.parse_qsl(b.decode()))
        assert form["Action"] == "AssumeRoleWithWebIdentity" and form["WebIdentityToken"] == "eyJhbGciOi.web.identity"
        assert form["RoleArn"] == "arn:aws:iam::123456789012:role/profile-ctl" and "Authorization" not in h
        return 200, ('<AssumeRoleWithWebIdentityResponse xmlns="https://sts.amazonaws.com/doc/2011-06-15/">'
                     '<AssumeRoleWithWebIdentityResult><Credentials><AccessKeyId>ASIATEMP</AccessKeyId>'
                     '<SecretAccessKey>tempsecret</SecretAccessKey><SessionToken>sess-tok</SessionToken>'
                     '<Expiration>2015-08-30T13:36:00Z</Expiration></Credentials>'
                     '</AssumeRoleWithWebIdentityResult></AssumeRoleWithWebIdentityResponse>')
    rec = Recorder([(lambda m, u, h, b: u == "https://sts.us-west-2.amazonaws.com/", sts)] + _aws_routes(state))
    env = {"AWS_ROLE_ARN": "arn:aws:iam::123456789012:role/profile-ctl", "AWS_WEB_IDENTITY_TOKEN_FILE": str(tok),
           "AWS_REGION": "us-west-2"}
    a = AwsIam(rec, env=env, clock=lambda: T0)
    a.aws_get_assume_role_policy("kf-user")
    a.aws_get_assume_role_policy("kf-user")
    assert sum(c["url"].startswith("https://sts.") for c in rec.calls) == 1, "STS credentials are cached"
    assert all(c["headers"].get("X-Amz-Security-Token") == "sess-tok" for c in rec.calls if "iam." in c["url"])


def test_no_aws_credentials_is_an_error(tmp_path):
    with pytest.raises(cloud_iam.CloudIamError):
        AwsCredentials(env={"AWS_SHARED_CREDENTIALS_FILE": str(tmp_path / "none")}).get()


# ------------------------------------------------------------------ end to end through the controller
def test_profile_plugins_drive_both_clouds():
    from service_account_auth_improvements_amd.controlplane import profile
    from service_account_auth_improvements_amd.controlplane.apiserver import APIServer
    from service_account_auth_improvements_amd.controlplane.client import InMemoryClient
    from service_account_auth_improvements_amd.controlplane.runtime import Manager
    gstore = {"p": {"bindings": []}}
    astate = {"doc": ROLE_DOC, "ak": "AKIDENV", "sk": "secretenv"}
    rec = Recorder(_gcp_routes(gstore) + _aws_routes(astate))
    backend = CloudIam(rec, env={"AWS_ACCESS_KEY_ID": "AKIDENV", "AWS_SECRET_ACCESS_KEY": "secretenv"})
    backend.aws.clock = lambda: T0
    c = InMemoryClient(APIServer())
    for cr in profile.default_cluster_roles():
        c.create(cr)
    mgr = Manager(c)
    mgr.add(profile.ProfileReconciler(c, iam=backend, ns_wait_s=0.0, labels_path="/nonexistent"))
    c.create({"apiVersion": "kubeflow.org/v1", "kind": "Profile", "metadata": {"name": "team-a"},
              "spec": {"owner": {"kind": "User", "name": "a@x.com"},
                       "plugins": [{"kind": "WorkloadIdentity",
                                    "spec": {"gcpServiceAccount": "kf-user@gcp-proj.iam.gserviceaccount.com"}},
                                   {"kind": "AwsIamForServiceAccount",
                                    "spec": {"awsIamRole": "arn:aws:iam::123456789012:role/kf-user"}}]}})
    mgr.run_until_idle()
    wi = [b for b in gstore["p"]["bindings"] if b["role"] == "roles/iam.workloadIdentityUser"]
    assert wi and wi[0]["members"] == ["serviceAccount:cluster-proj.svc.id.goog[team-a/default-editor]"]
    cond = astate["doc"]["Statement"][0]["Condition"]["StringEquals"]
    assert cond["oidc.eks.us-west-2.amazonaws.com/id/ABC:sub"] == ["system:serviceaccount:team-a:default-editor"]
    sa = c.get("v1", "ServiceAccount", "default-editor", "team-a")
    assert sa["metadata"]["annotations"]["eks.amazonaws.com/role-arn"] == "arn:aws:iam::123456789012:role/kf-user"
    # delete -> both plugins revoke
    c.delete("kubeflow.org/v1", "Profile", "team-a")
    mgr.run_until_idle()
    assert all("team-a" not in m for b in gstore["p"]["bindings"] for m in b["members"])
    assert "oidc.eks.us-west-2.amazonaws.com/id/ABC:sub" not in astate["doc"]["Statement"][0]["Condition"]["StringEquals"]
    mgr.stop()
