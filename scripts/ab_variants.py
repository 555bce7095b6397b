"""Same-box A/B of kernel-source variants: build each variant of the package into its own tree
under `ab/<name>/` (package + scripts, its own `_C` extension), and write `ab/run.sh`, which runs
one timing command per variant in interleaved passes on the GPU box.  Boxes differ by 1-2 %
(profiles/r4v_flush_vector_publish_ab.txt: the same HEAD measured 150.3 and 151.1-152.0 us on
two boxes), so a variant is only ever compared with the others of the same call.

    python scripts/ab_variants.py \
        --variant base \
        --variant keep16 'splitlearning_amd/csrc/hybrid.hip|constexpr int kKeepM = 7;|constexpr int kKeepM = 15;' \
        --cmd 'python -u {root}/scripts/hybrid_ab.py --tp 1 --steps 500 --rounds 3 --only hybrid' --passes 2
    gpurun --timeout 900 -- 'mkdir -p gpurun_out && bash ab/run.sh'   # -> gpurun_out/ab.log

Each substitution is FILE|OLD|NEW (OLD must occur in FILE; every occurrence is replaced) or
FILE<SRC (the variant's FILE becomes a copy of SRC, e.g. a saved earlier version of a kernel).  The
timing command runs with `{root}` = the variant's tree, whose scripts put that tree first on
sys.path.  `ab/` is git-ignored; delete it after the call (it ships with every gpurun call).
"""
import argparse
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build_variant(out, name, subs):
    root = os.path.join(out, name)
    shutil.rmtree(root, ignore_errors=True)
    os.makedirs(root)
    for d in ("splitlearning_amd", "scripts"):
        shutil.copytree(os.path.join(REPO, d), os.path.join(root, d),
                        ignore=shutil.ignore_patterns("__pycache__", "build"))
    for spec in subs:
        if "<" in spec and "|" not in spec:     # FILE<SRC: the variant's FILE is a copy of SRC
            path, src = spec.split("<", 1)
            shutil.copyfile(src, os.path.join(root, path))
            continue
        path, old, new = spec.split("|", 2)
        p = os.path.join(root, path)
        with open(p) as f:
            s = f.read()
        if old not in s:
            sys.exit(f"{name}: '{old}' not found in {path}")
        with open(p, "w") as f:
            f.write(s.replace(old, new))
    r = subprocess.run([sys.executable, "-c", "from splitlearning_amd import build as b; b.build()"],
                       cwd=root, capture_output=True, text=True)
    if r.returncode != 0:
        sys.exit(f"{name}: build failed\n{r.stderr[-3000:]}")
    shutil.rmtree(os.path.join(root, "splitlearning_amd", "build"), ignore_errors=True)
    return root


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", nargs="+", action="append", required=True, metavar="NAME [FILE|OLD|NEW ...]")
    ap.add_argument("--cmd", required=True)
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--timeout", type=int, default=150, help="seconds per timing run")
    ap.add_argument("--out", default=os.path.join(REPO, "ab"))
    a = ap.parse_args()
    names = []
    for v in a.variant:
        build_variant(a.out, v[0], v[1:])
        names.append(v[0])
        print(f"built {v[0]}", flush=True)
    rel = os.path.relpath(a.out, REPO)
    lines = ["set -e", f"for r in $(seq {a.passes}); do", f"for v in {' '.join(names)}; do",
             '  echo "== $v" >> gpurun_out/ab.log',
             f"  timeout -k 10 {a.timeout} {a.cmd.format(root=rel + '/$v')} >> gpurun_out/ab.log 2>&1",
             "done", "done"]
    with open(os.path.join(a.out, "run.sh"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print(f"wrote {rel}/run.sh", flush=True)


if __name__ == "__main__":
    main()
