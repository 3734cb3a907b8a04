"""Timing-only variant builds of libgr.so from a patched copy of the sources (the product sources carry no
ablation switches).  A patch is a JSON list of [file, old, new] text replacements; every `old` must occur
exactly once; {"rev": COMMIT} builds that commit's sources instead of the tree's.  Output: variants/<name>/libgr.so
(GR_LIB_PATH selects it on the GPU box).

    python scripts/build_patched.py NAME PATCH.json [-DMACRO=VALUE ...]

Extra arguments are passed to hipcc (cache-policy macros such as -DGR_STATE_STORE_POLICY=0); PATCH.json may be `-`
for no text replacements.
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(name, patch, extra_flags="", rev=None):
    tmp = tempfile.mkdtemp(prefix="grvar_")
    src = os.path.join(tmp, "generalizableracing_amd", "csrc")
    if rev:  # the sources of an earlier commit (a before / after pair on the same box)
        subprocess.run(f"git -C {ROOT} archive {rev} generalizableracing_amd/csrc include | tar -x -C {tmp}", shell=True,
                       check=True)
    else:
        shutil.copytree(os.path.join(ROOT, "generalizableracing_amd", "csrc"), src)
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    for fname, old, new in patch:
        p = os.path.join(src, fname)
        s = open(p).read()
        if s.count(old) != 1:
            raise SystemExit(f"{fname}: patch text found {s.count(old)} times: {old[:80]!r}")
        open(p, "w").write(s.replace(old, new))
    out = os.path.join(ROOT, "variants", name)
    os.makedirs(out, exist_ok=True)
    flags = ("--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt "
             "-fno-slp-vectorize " + extra_flags)
    objs = []
    for f in ("gr_kernels.hip", "gr_camera.hip", "gr_policy.hip", "gr_policy_f32.hip", "gr_bn.hip", "gr_update.hip",
              "gr_mlp.hip", "gr_rollout.hip", "gr_terrain.hip", "gr_capi.cpp"):
        o = os.path.join(tmp, f + ".o")
        extra = " -fno-honor-nans" if f == "gr_policy.hip" else ""
        lang = " -x hip" if f.endswith(".cpp") else ""
        subprocess.run(f"/opt/rocm/bin/hipcc {flags}{extra}{lang} -c -o {o} {os.path.join(src, f)}", shell=True, check=True)
        objs.append(o)
    subprocess.run(f"/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o {out}/libgr.so {' '.join(objs)}", shell=True,
                   check=True)
    shutil.rmtree(tmp)
    print(f"{out}/libgr.so")


def load_patch(path):
    """A patch file: a JSON list of [file, old, new] replacements, or {"replace": [...], "flags": "-D...",
    "note": "..."} (variants/patches/*.json)."""
    if path == "-":
        return [], "", None
    p = json.load(open(path))
    if isinstance(p, dict):
        return p.get("replace", []), p.get("flags", ""), p.get("rev")
    return p, "", None


if __name__ == "__main__":
    reps, flags, rev = load_patch(sys.argv[2])
    build(sys.argv[1], reps, " ".join([flags] + sys.argv[3:]), rev)
