"""Generate the per-component GitHub Actions workflows (P6; the reference keeps one set per
component under .github/workflows: ``<component>_unit_test.yaml``, ``*_intergration_test.yaml``,
``*_docker_publish.yaml``, e.g. nb_controller_intergration_test.yaml, jwa_backend_unittests.yaml).

Each component gets, triggered by changes under its paths:
* ``<id>_unit_test.yaml`` -- its unit tests (CPU);
* ``<id>_integration_test.yaml`` -- its image build plan, then ``tools/ci_integration.py <id>``
  against the multi-process cluster (apiserver / controller-manager / kubelet over HTTP), the
  stand-in for the reference's KinD deploy-and-wait jobs;
* ``<id>_docker_publish.yaml`` -- build and push its image on main;
* ``<id>_multi_arch_test.yaml`` -- for the control-plane components (no GPU runtime in their
  image): build it for linux/amd64, linux/ppc64le and linux/arm64/v8 under QEMU + buildx, as the
  reference's ``*_multi_arch_test.yaml`` do.  The ROCm notebook / trainer / predictor images
  target MI355X hosts and stay linux/amd64.

  python tools/gen_workflows.py            # (re)write .github/workflows/<id>_*.yaml
  python tools/gen_workflows.py --check    # exit 1 if any generated file is stale
"""
from __future__ import annotations

import argparse
import os
import sys

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, ".github", "workflows")
PKG = "service_account_auth_improvements_amd"
IMAGE = "rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.10.0"

# id -> (workflow title, source paths, unit-test selection, image, tools/ci_integration.py component)
COMPONENTS = {
    "notebook_controller": ("Notebook Controller", [f"{PKG}/controlplane/notebook.py",
                                                    f"{PKG}/runtime/notebook_server.py"],
                            "tests/test_notebook_controller.py tests/test_notebook_server.py", "platform",
                            "notebook-controller"),
    "profile_controller": ("Profile Controller + KFAM",
                           [f"{PKG}/controlplane/profile.py", f"{PKG}/controlplane/kfam.py",
                            f"{PKG}/controlplane/cloud_iam.py", f"{PKG}/controlplane/monitoring.py"],
                           "tests/test_controllers.py -k profile tests/test_kfam.py tests/test_cloud_iam.py",
                           "platform", "profile-controller"),
    "poddefaults": ("PodDefaults Webhook", [f"{PKG}/controlplane/poddefault.py"],
                    "tests/test_controllers.py -k poddefault", "platform", "poddefaults"),
    "tb_controller": ("Tensorboard Controller", [f"{PKG}/controlplane/tensorboard.py"],
                      "tests/test_controllers.py -k tensorboard", "platform", "tensorboard-controller"),
    "pvcviewer_controller": ("PVCViewer Controller", [f"{PKG}/controlplane/pvcviewer.py"],
                             "tests/test_controllers.py -k pvcviewer", "platform", "pvcviewer-controller"),
    "training_operator": ("Training Operator (PyTorchJob / MPIJob)",
                          [f"{PKG}/controlplane/training.py", f"{PKG}/controlplane/mpi.py", f"{PKG}/native/**"],
                          "tests/test_training_operator.py tests/test_mpijob.py tests/test_native_sanitize.py",
                          "platform",
                          "training-operator"),
    "jwa": ("Jupyter Web App", [f"{PKG}/webapps/jupyter.py", f"{PKG}/webapps/crud_backend.py",
                                f"{PKG}/webapps/config/**"],
            "tests/test_webapps.py -k 'jwa or authn or authz or uptime or form or status'", "platform",
            "jupyter-web-app"),
    "vwa": ("Volumes Web App", [f"{PKG}/webapps/volumes.py", f"{PKG}/webapps/crud_backend.py"],
            "tests/test_webapps.py -k vwa", "platform", "volumes-web-app"),
    "twa": ("Tensorboards Web App", [f"{PKG}/webapps/tensorboards.py", f"{PKG}/webapps/crud_backend.py"],
            "tests/test_webapps.py -k twa", "platform", "tensorboards-web-app"),
    "centraldb": ("Central Dashboard", [f"{PKG}/webapps/dashboard.py", f"{PKG}/webapps/static/**"],
                  "tests/test_dashboard.py tests/test_ui.py", "platform", "centraldashboard"),
}


def _on(paths):
    return {"pull_request": {"paths": paths + ["tools/ci_integration.py", "tools/gen_workflows.py"],
                             "branches": ["main"]},
            "push": {"paths": paths, "branches": ["main"]}}


def _checkout():
    return [{"uses": "actions/checkout@v4"}]


def workflows():
    out = {}
    for cid, (title, paths, tests, image, integ) in COMPONENTS.items():
        conc = {"group": "${{ github.workflow }}-${{ github.ref }}", "cancel-in-progress": True}
        out[f"{cid}_unit_test.yaml"] = {
            "name": f"{title} Unit Test", "on": _on(paths + [t for t in tests.split() if t.startswith("tests/")]),
            "concurrency": conc,
            "jobs": {"unit": {"runs-on": "ubuntu-22.04", "container": IMAGE, "steps": _checkout() + [
                {"name": "build native parts", "run": "python3 -c \"from service_account_auth_improvements_amd."
                                                      "native import build_native; build_native()\""},
                {"name": "unit tests", "run": f"python3 -m pytest -q {tests}"}]}}}
        out[f"{cid}_integration_test.yaml"] = {
            "name": f"{title} Integration Test", "on": _on(paths), "concurrency": conc,
            "jobs": {"integration": {"runs-on": "ubuntu-22.04", "container": IMAGE, "steps": _checkout() + [
                {"name": "image build plan", "run": f"python3 tools/build_images.py --dry-run {image}"},
                {"name": "multi-process cluster + sample",
                 "run": f"timeout 600 python3 tools/ci_integration.py {integ}"}]}}}
        out[f"{cid}_docker_publish.yaml"] = {
            "name": f"{title} Docker Publish", "on": {"push": {"paths": paths, "branches": ["main"]}},
            "jobs": {"publish": {"runs-on": "ubuntu-22.04", "steps": _checkout() + [
                {"name": "build and push",
                 "run": f"python3 tools/build_images.py {image} --registry ghcr.io/${{{{ github.repository_owner }}}} "
                        "--tag ${{ github.sha }} --push"}]}}}
    for cid, (title, paths, tests, image, integ) in COMPONENTS.items():
        if image != "platform":
            continue
        out[f"{cid}_multi_arch_test.yaml"] = {
            "name": f"{title} Multi-Arch Build Test",
            "on": {"pull_request": {"paths": paths + ["images/platform/**"], "branches": ["main"]}},
            "concurrency": {"group": "${{ github.workflow }}-${{ github.ref }}-${{ github.event.number }}",
                            "cancel-in-progress": True},
            "jobs": {"build": {"runs-on": "ubuntu-22.04", "steps": _checkout() + [
                {"name": "Setup QEMU", "uses": "docker/setup-qemu-action@v3"},
                {"name": "Setup Docker Buildx", "uses": "docker/setup-buildx-action@v3"},
                {"name": "Build multi-arch image",
                 "run": "python3 tools/build_images.py platform --platforms "
                        "linux/amd64,linux/ppc64le,linux/arm64/v8"}]}}}
    out["example_notebook_servers_publish.yaml"] = {
        "name": "Example Notebook Servers Publish", "on": {"push": {"paths": ["images/**"], "branches": ["main"]}},
        "jobs": {"publish": {"runs-on": "ubuntu-22.04", "steps": _checkout() + [
            {"name": "build and push every notebook image (dependency order)",
             "run": "python3 tools/build_images.py --registry ghcr.io/${{ github.repository_owner }} "
                    "--tag ${{ github.sha }} --push"}]}}}
    out["common_frontend_tests.yaml"] = {
        "name": "Common Frontend Tests", "on": _on([f"{PKG}/webapps/static/**", "tests/js/**"]),
        "jobs": {"frontend": {"runs-on": "ubuntu-22.04", "steps": _checkout() + [
            {"uses": "actions/setup-node@v4", "with": {"node-version": "20"}},
            {"name": "syntax + logic tests", "run": "node tests/js/kf_logic_cases.js"}]}}}
    out["python_lint.yaml"] = {
        "name": "Python Lint", "on": {"pull_request": {"paths": ["**.py"], "branches": ["main"]}},
        "jobs": {"lint": {"runs-on": "ubuntu-22.04", "steps": _checkout() + [
            {"uses": "actions/setup-python@v5", "with": {"python-version": "3.10"}},
            {"name": "byte-compile everything", "run": f"python -m compileall -q {PKG} tools tests bench.py"}]}}}
    return out


HEADER = "# Generated by tools/gen_workflows.py -- edit the generator, not this file.\n"


def render(doc) -> str:
    # PyYAML writes the key `on` as `'on'`; GitHub accepts either
    return HEADER + yaml.safe_dump(doc, sort_keys=False, width=120)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args(argv)
    stale = []
    os.makedirs(OUT, exist_ok=True)
    for name, doc in workflows().items():
        path = os.path.join(OUT, name)
        text = render(doc)
        cur = open(path).read() if os.path.exists(path) else None
        if cur != text:
            stale.append(name)
            if not a.check:
                with open(path, "w") as f:
                    f.write(text)
    if a.check and stale:
        print("stale workflows:", " ".join(stale))
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
