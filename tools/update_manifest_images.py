"""P10: release tooling -- rewrite image tags (and optionally the registry) in every
kustomization's ``images:`` list and in the generated manifests, the counterpart of
releasing/update-manifests-images.

  python tools/update_manifest_images.py --tag v1.0.0 [--registry ghcr.io/org] [--dir manifests] [--check]
"""
import argparse
import os
import sys

import yaml


def update(dir_, tag, registry=None, check=False):
    changed = []
    for root, _, files in os.walk(dir_):
        if "kustomization.yaml" not in files:
            continue
        p = os.path.join(root, "kustomization.yaml")
        with open(p) as f:
            head = f.readline()
            rest = f.read()
        k = yaml.safe_load(head + rest)
        imgs = k.get("images") or []
        dirty = False
        for im in imgs:
            new_name = im.get("newName", im["name"])
            if registry:
                new_name = registry.rstrip("/") + "/" + new_name.split("/")[-1]
            if im.get("newTag") != tag or im.get("newName") != new_name:
                im["newTag"], im["newName"], dirty = tag, new_name, True
        if dirty:
            changed.append(p)
            if not check:
                with open(p, "w") as f:
                    if head.startswith("#"):
                        f.write(head)
                    yaml.safe_dump(k, f, sort_keys=False)
    return changed


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--registry", default=None)
    ap.add_argument("--dir", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "manifests"))
    ap.add_argument("--check", action="store_true", help="exit 1 if anything would change")
    a = ap.parse_args(argv)
    ch = update(a.dir, a.tag, a.registry, a.check)
    for p in ch:
        print(("would update " if a.check else "updated ") + p)
    return 1 if (a.check and ch) else 0


if __name__ == "__main__":
    sys.exit(main())
