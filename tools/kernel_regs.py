"""Per-kernel register / spill / LDS table of one HIP source compiled for gfx950 (hipcc
-Rpass-analysis=kernel-resource-usage), for comparing a change against a committed revision.

    python tools/kernel_regs.py image_recommender_amd/csrc/knn_i8.hip [--rev HEAD] [--filter scan]

--rev: compile the file (and the csrc headers) as of that git revision instead of the worktree.
"""
import argparse
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "image_recommender_amd", "csrc")


def table(src: str, inc: str):
    with tempfile.TemporaryDirectory() as td:
        r = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + inc, "-c", src,
                            "-o", os.path.join(td, "k.o"), "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True, cwd=td)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(?:Function Name: (\S+)|(\w[\w ]*?)(?: \[[^\]]*\])?: (\d+))", line)
        if not m:
            continue
        if m.group(1):
            cur = {"name": m.group(1)}
            rows.append(cur)
        elif cur is not None:
            cur[m.group(2).strip()] = int(m.group(3))
    if r.returncode != 0:
        raise SystemExit(r.stderr[-3000:])
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--rev", default=None)
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    src, inc = os.path.abspath(a.src), CSRC
    td = None
    if a.rev:
        td = tempfile.mkdtemp()
        rel = os.path.relpath(CSRC, ROOT)
        for f in subprocess.run(["git", "ls-tree", "--name-only", a.rev, rel + "/"], cwd=ROOT,
                                capture_output=True, text=True, check=True).stdout.split():
            with open(os.path.join(td, os.path.basename(f)), "w") as fh:
                fh.write(subprocess.run(["git", "show", f"{a.rev}:{f}"], cwd=ROOT, capture_output=True,
                                        text=True, check=True).stdout)
        src, inc = os.path.join(td, os.path.basename(a.src)), td
    for r in table(src, inc):
        if a.filter not in r["name"]:
            continue
        print(f"{r.get('VGPRs', '?'):>4} v {r.get('AGPRs', '?'):>4} a  spill s {r.get('SGPRs Spill', '?'):>3}"
              f" v {r.get('VGPRs Spill', '?'):>3}  lds {r.get('LDS Size', '?'):>6}  {r['name'][:110]}")


if __name__ == "__main__":
    main()
