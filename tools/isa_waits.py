#!/usr/bin/env python3
"""Where does a sweep kernel wait for memory?  Compiles a HIP source for gfx950 to assembly (no GPU
needed) and lists, per loop of one kernel, the `s_waitcnt vmcnt(N)` with small N -- a wait that
lets only N memory operations stay in flight, i.e. (nearly) a whole round trip -- plus waterfall
loops (`s_and_saveexec` around a buffer access whose SGPR offset the compiler could not prove
uniform) and scratch use.  The ring waits of the pair sweep are vmcnt(24/25) (single-run) and
vmcnt(48-51) (generic); anything far below those inside a chunk loop is a stall per chunk.

    python tools/isa_waits.py [--src large-scale-recommendation_amd/csrc/kernels_pair.hip]
                              [--kernel 'k_sweep_pair_sysILi2ELi7'] [--below 16] [--keep out.s]

Found with it (round 4): the k=128 generic loop's chunk loads were a
readfirstlane waterfall followed by vmcnt(0) at every 56-pair chunk boundary.
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "large-scale-recommendation_amd", "csrc")


def compile_asm(src, out):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
           "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "--cuda-device-only", "-S", "-o", out, src]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)


def kernel_body(lines, name):
    """The assembly lines of the kernel with this mangled name (label to s_endpgm)."""
    for i, l in enumerate(lines):
        if l.startswith(name + ":"):
            j = i
            while j < len(lines) and "s_endpgm" not in lines[j]:
                j += 1
            return lines[i:j + 1]
    return []


def loop_report(body, below):
    """{loop header label: (lines, buffer ops, [small vmcnt values])} for every loop of depth >= 2,
    by the assembler's 'in Loop: Header=' annotations."""
    loops, order, cur = {}, [], None
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):\s*;\s*(.*)", l)
        if m:
            cur = None
            mh = re.search(r"Header=BB(\d+_\d+) Depth=(\d+)", m.group(2))
            nxt = body[i + 1] if i + 1 < len(body) else ""
            if mh and int(mh.group(2)) >= 2:
                cur = mh.group(1)
            elif "Loop Header: Depth=" in nxt and int(re.search(r"Depth=(\d+)", nxt).group(1)) >= 2:
                cur = m.group(1).replace(".LBB", "")
            if cur is not None and cur not in loops:
                loops[cur] = [0, 0, []]
                order.append(cur)
            continue
        if cur is None:
            continue
        st = loops[cur]
        st[0] += 1
        if re.search(r"buffer_(load|store)", l):
            st[1] += 1
        w = re.search(r"s_waitcnt vmcnt\((\d+)\)", l)
        if w and int(w.group(1)) < below:
            st[2].append(int(w.group(1)))
    return [(k, *loops[k]) for k in order]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(CSRC, "kernels_pair.hip"))
    ap.add_argument("--kernel", default="k_sweep_pair_sys")
    ap.add_argument("--below", type=int, default=16)
    ap.add_argument("--keep", default=None, help="also write the assembly here")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        out = a.keep or os.path.join(td, "k.s")
        compile_asm(a.src, out)
        lines = open(out).read().splitlines()
    names = sorted({m.group(1) for l in lines for m in [re.match(r"^(_Z\S*" + a.kernel + r"\S*):", l)] if m})
    if not names:
        sys.exit(f"no kernel matching {a.kernel}")
    for name in names:
        body = kernel_body(lines, name)
        waterfalls = sum("s_and_saveexec" in l for l in body)
        scratch = sum("scratch_" in l for l in body)
        print(f"{name}: {len(body)} lines, {waterfalls} s_and_saveexec, {scratch} scratch ops")
        for hdr, n, ops, small in loop_report(body, a.below):
            if ops:
                print(f"  loop BB{hdr}: {n} lines, {ops} buffer ops, vmcnt < {a.below}: {small}")


if __name__ == "__main__":
    main()
