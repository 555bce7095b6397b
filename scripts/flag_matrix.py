"""Robustness sweep on one GPU: every mode under a matrix of framework flags, through the
real launcher (small synthetic data).  Prints one line per run: PASS/FAIL, seconds, flags.

    python scripts/flag_matrix.py [--out gpurun_out/flag_matrix.txt]
"""
import argparse
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODES = [["--sisa"], ["--vanilla"], [], ["--sisa", "--concat", "--concat_unlearn"], ["--control"]]
EXTRAS = [[], ["--dtype", "bf16"], ["--act_dtype", "bf16"], ["--batch_size", "32"], ["--batch_size", "64"],
          ["--graphs", "on"], ["--graphs", "off"], ["--python_epoch"], ["--world_size", "5"],
          ["--kernels", "torch"], ["--serial_alices", "--world_size", "4"], ["--true_reset", "--eval_dropout_fix"]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    lines, fails = [], 0
    for mode in MODES:
        for extra in EXTRAS:
            with tempfile.TemporaryDirectory() as d:
                argv = [sys.executable, os.path.join(ROOT, "split_nn.py")] + mode + [
                    "--iterations", "1", "--server_epochs", "1", "--num_samples", "3000", "--seed", "1",
                    "--no_tqdm", "--device", "cuda", "--datapath", os.path.join(d, "data"),
                    "--log_dir", os.path.join(d, "logs")]
                if "--world_size" not in extra:
                    argv += ["--world_size", "3"]
                argv += extra
                t0 = time.time()
                r = subprocess.run(argv, capture_output=True, text=True, timeout=300, cwd=ROOT)
                dt = time.time() - t0
                ok = r.returncode == 0
                fails += not ok
                line = f"{'PASS' if ok else 'FAIL'} {dt:6.1f}s {' '.join(mode + extra) or '(U-shape)'}"
                if not ok:
                    line += "\n    " + "\n    ".join((r.stderr or r.stdout).strip().splitlines()[-6:])
                print(line, flush=True)
                lines.append(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + f"\n{fails} failed of {len(lines)}\n")
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
