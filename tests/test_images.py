"""Notebook server images (I1): the reference's image set has a counterpart here (CUDA flavours
replaced by ROCm), the Dockerfiles chain as the builder says, the spawner only offers images
this repo builds, and the container init (kf-entrypoint + cont-init scripts) behaves like the
reference's s6 ``01-copy-tmp-home``."""
import os
import re
import stat
import subprocess
import sys

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import build_images  # noqa: E402

# components/example-notebook-servers/Makefile:1-17 (IMAGE_FOLDERS, build order)
REFERENCE_IMAGES = ["base", "codeserver", "codeserver-python", "jupyter", "jupyter-scipy", "jupyter-pytorch",
                    "jupyter-pytorch-full", "jupyter-pytorch-cuda", "jupyter-pytorch-cuda-full", "jupyter-tensorflow",
                    "jupyter-tensorflow-full", "jupyter-tensorflow-cuda", "jupyter-tensorflow-cuda-full", "rstudio",
                    "rstudio-tidyverse"]


def test_every_reference_image_has_a_counterpart():
    for name in REFERENCE_IMAGES:
        ours = name.replace("-cuda", "-rocm")
        assert ours in build_images.IMAGES, ours
        assert os.path.exists(os.path.join(ROOT, build_images.IMAGES[ours][1]))
    assert len(build_images.NOTEBOOK_IMAGES) >= len(REFERENCE_IMAGES)


def test_dockerfile_bases_match_the_builder_dependencies():
    for name, (ctx, df, args, deps) in build_images.IMAGES.items():
        text = open(os.path.join(ROOT, df)).read()
        for k, v in args.items():
            m = re.search(rf"^ARG {k}=(\S+)", text, re.M)
            assert m, (name, k)
            dep = v.format(r="kfamd", t="latest")
            assert m.group(1) == dep, (name, m.group(1), dep)
            assert dep.split("/")[1].split(":")[0] in deps, (name, dep)
        for f in re.findall(r"^COPY (?!--from)(\S+)", text, re.M):
            assert os.path.exists(os.path.join(ROOT, ctx, f.rstrip("/"))), (name, f)
    order = build_images.order(list(build_images.IMAGES))
    for name, (_, _, _, deps) in build_images.IMAGES.items():
        assert all(order.index(d) < order.index(name) for d in deps)


def test_spawner_offers_only_built_images():
    cfg = yaml.safe_load(open(os.path.join(ROOT, "service_account_auth_improvements_amd", "webapps", "config",
                                           "spawner_ui_config.yaml")))["spawnerFormDefaults"]
    for key in ("image", "imageGroupOne", "imageGroupTwo"):
        for img in [cfg[key]["value"]] + cfg[key]["options"]:
            name = img.split("/")[1].split(":")[0]
            assert img.startswith("kfamd/") and name in build_images.NOTEBOOK_IMAGES, img


def _exe(path, text):
    path.write_text(text)
    path.chmod(path.stat().st_mode | stat.S_IXUSR)


def test_copy_tmp_home_and_entrypoint(tmp_path):
    home, tmp_home, init = tmp_path / "home", tmp_path / "tmp_home", tmp_path / "init.d"
    home.mkdir()
    (tmp_home / ".jupyter").mkdir(parents=True)
    (tmp_home / ".jupyter" / "settings.json").write_text("default")
    (tmp_home / ".jupyter").chmod(0o775)
    (tmp_home / "keep.txt").write_text("from image")
    (home / "keep.txt").write_text("user data")           # an existing file on the PVC is never overwritten
    init.mkdir()
    src = open(os.path.join(ROOT, "images", "base", "init", "cont-init.d", "01-copy-tmp-home")).read()
    _exe(init / "01-copy-tmp-home", src)
    _exe(init / "05-mark", "#!/bin/bash\necho marker > \"$HOME/.initialised\"\n")
    env = dict(os.environ, HOME=str(home), HOME_TMP=str(tmp_home), KF_INIT_DIR=str(init))
    r = subprocess.run(["bash", os.path.join(ROOT, "images", "base", "init", "kf-entrypoint"), "bash", "-c",
                        "echo started:$(cat $HOME/.initialised)"], capture_output=True, text=True, env=env, timeout=30)
    assert r.returncode == 0, r.stderr
    assert "started:marker" in r.stdout and "init 01-copy-tmp-home" in r.stdout
    assert (home / ".jupyter" / "settings.json").read_text() == "default"
    assert (home / "keep.txt").read_text() == "user data"
    assert (home / ".jupyter").stat().st_mode & stat.S_IWGRP       # umask 0002 keeps it group-writable


def test_failing_init_script_aborts_start(tmp_path):
    init = tmp_path / "init.d"
    init.mkdir()
    _exe(init / "01-fail", "#!/bin/bash\nexit 3\n")
    env = dict(os.environ, KF_INIT_DIR=str(init))
    r = subprocess.run(["bash", os.path.join(ROOT, "images", "base", "init", "kf-entrypoint"), "echo", "never"],
                       capture_output=True, text=True, env=env, timeout=30)
    assert r.returncode != 0 and "never" not in r.stdout
