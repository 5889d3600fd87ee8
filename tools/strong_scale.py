"""Strong-scaling harness (the GPU counterpart of the
reference's multigrid_strongsc.cpp thread sweep): runs bench.py at N=16384 on
G = 1, 2, 4, 8 GPUs (torch.distributed.run for G > 1, only G <= visible GPUs)
and writes strong_scale.txt as "%d\t%f\n" (G, seconds per V-cycle), the
format strongsc_plot.py reads, plus the JSON lines to strong_scale.jsonl.
    python tools/strong_scale.py [--gpus 1,2,4,8] [--steps 20] [--N 16384 --levels 9]"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--N", type=int, default=16384)
    ap.add_argument("--levels", type=int, default=9)
    ap.add_argument("--out", default="strong_scale.txt")
    a = ap.parse_args()
    import torch
    avail = torch.cuda.device_count()
    common = ["--steps", str(a.steps), "--warmup", str(a.warmup), "--N", str(a.N),
              "--levels", str(a.levels), "--cpu-baseline", "off", "--no-profile"]
    rows = []
    for g in (int(x) for x in a.gpus.split(",")):
        if g > avail:
            print(f"skip G={g}: {avail} GPU(s) visible", flush=True)
            continue
        if g == 1:
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"] + common
        else:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   f"--nproc-per-node={g}", "--master-addr", "127.0.0.1",
                   "--master-port", str(29400 + g), os.path.join(ROOT, "bench.py"),
                   "--gpus", str(g)] + common
        out = subprocess.run(cmd, capture_output=True, text=True, check=True).stdout
        line = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
        rows.append((g, line["ms_per_step"] / 1e3, line))
        print(f"G={g}: {line['ms_per_step']:.3f} ms/V-cycle, {line['value']:.3e} GPUPS",
              flush=True)
    with open(a.out, "w") as f:
        for g, s, _ in rows:
            f.write("%d\t%f\n" % (g, s))
    with open(os.path.splitext(a.out)[0] + ".jsonl", "w") as f:
        for _, _, line in rows:
            f.write(json.dumps(line) + "\n")


if __name__ == "__main__":
    main()
