#!/usr/bin/env python3
"""Static checks of the gfx950 machine code in the BUILT libmfhip.so (no GPU needed).

The .so's `.hip_fatbin` section holds one clang offload bundle per kernel source; every
gfx950 code object is extracted and disassembled with llvm-objdump, and each kernel is turned
into a control-flow graph (fall-through + branch targets).  Two checks run on it:

1. Store-data hazard.  A vector-memory store of more than 64 bits (`*_store_dwordx3/x4`) reads
   its data VGPRs after it issues; a VALU that overwrites them too soon corrupts the stored
   value.  The hazard table asks for 1 wait state and exempts `buffer_store` with an SGPR
   `soffset`; LLVM's hazard recognizer follows that exemption (GCNHazardRecognizer::
   createsVALUHazard) and pads nothing there.  On gfx950 the exemption does not hold
   (tools/micro/store_data_hazard.hip, profiles/r05_store_data_hazard.txt): the round-4 k = 256
   lean sweep, whose compiled code overwrote b128 store data one or two instructions after the
   store, was the only build that did not repeat itself.  `store_hazards` finds every store of
   more than 64 bits followed, on any path, by a VALU write of its data VGPRs within `ws` wait
   states (each instruction is one, `s_nop N` is N + 1).

2. Hand-counted hand-off waits.  A progress or ticket word may be stored only after the stores
   it publishes have landed; the kernels wait with hand-counted `s_waitcnt vmcnt(N)` (the N
   youngest operations may still fly).  `flag_store_violations` walks back from every flag
   store over every path: no row store may sit between the wait and the flag store, and the N
   operations younger than the wait may hold a row store only where the protocol allows it --
   mode "all" (systolic sweep: none at all) or "prev" (ticket sweeps that publish an entry's
   ticket one or two entries late: only stores issued after the previous flag store, i.e. of
   entries whose tickets are still held back).

    python tools/isa_check.py [--lib large-scale-recommendation_amd/lib/libmfhip.so]
"""
import argparse
import os
import re
import struct
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
DEFAULT_LIB = os.path.join(ROOT, "large-scale-recommendation_amd", "lib", "libmfhip.so")
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib):
    """The gfx950 ELF code objects of a HIP shared library (bytes each)."""
    out = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "-S", "-W", lib], check=True, capture_output=True,
                         text=True).stdout
    sec = None
    for line in out.splitlines():
        if ".hip_fatbin" in line:
            f = line.split("]", 1)[1].split()
            sec = (int(f[3], 16), int(f[4], 16))
    if sec is None:
        raise RuntimeError(f"{lib}: no .hip_fatbin section")
    with open(lib, "rb") as fh:
        fh.seek(sec[0])
        data = fh.read(sec[1])
    objs, pos = [], 0
    while True:
        p = data.find(BUNDLE_MAGIC, pos)
        if p < 0:
            break
        n = struct.unpack_from("<Q", data, p + 24)[0]
        q = p + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, q)
            q += 24
            triple = data[q:q + tlen].decode()
            q += tlen
            if triple.endswith("gfx950"):
                objs.append(data[p + off:p + off + size])
        pos = p + len(BUNDLE_MAGIC)
    return objs


class Ins:
    __slots__ = ("addr", "mn", "ops", "target", "idx")

    def __init__(self, addr, mn, ops, target):
        self.addr, self.mn, self.ops, self.target = addr, mn, ops, target


_FUNC = re.compile(r"^([0-9a-f]+) <(\S+)>:$")
_INS = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):[^<]*(?:<(\S+?)(?:\+0x([0-9a-f]+))?>)?\s*$")


def kernels(lib=DEFAULT_LIB):
    """{mangled kernel name: [Ins]} over every gfx950 code object of the library."""
    res = {}
    with tempfile.TemporaryDirectory() as td:
        for n, blob in enumerate(code_objects(lib)):
            path = os.path.join(td, f"co{n}.o")
            with open(path, "wb") as fh:
                fh.write(blob)
            dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", path], check=True,
                                 capture_output=True, text=True).stdout
            cur, start, body = None, 0, []
            for line in dis.splitlines():
                m = _FUNC.match(line)
                if m:
                    if cur:
                        res[cur] = body
                    cur, start, body = m.group(2), int(m.group(1), 16), []
                    continue
                m = _INS.match(line)
                if not m or cur is None:
                    continue
                tgt = None
                if m.group(4) is not None and m.group(1).startswith("s_") and "branch" in m.group(1):
                    tgt = start + (int(m.group(5), 16) if m.group(5) else 0)
                body.append(Ins(int(m.group(3), 16), m.group(1), m.group(2), tgt))
            if cur:
                res[cur] = body
    for body in res.values():
        for i, x in enumerate(body):
            x.idx = i
    return res


def successors(body, i, by_addr):
    x = body[i]
    if x.mn in ("s_endpgm", "s_setpc_b64", "s_trap"):
        return []
    if x.mn == "s_branch":
        return [by_addr[x.target]]
    nxt = [i + 1] if i + 1 < len(body) else []
    if x.mn.startswith("s_cbranch"):
        # an exec-zero skip is never taken by these kernels (lane 0 is active on every guarded path)
        if x.mn == "s_cbranch_execz":
            return nxt
        return nxt + [by_addr[x.target]]
    return nxt


def _regs(tok):
    m = re.match(r"^([va])\[(\d+):(\d+)\]$", tok)
    if m:
        return {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"^([va])(\d+)$", tok)
    return {(m.group(1), int(m.group(2)))} if m else set()


def _operands(ops):
    return [t.strip() for t in ops.split(",")] if ops else []


def is_vmem(mn):
    return mn.startswith(("buffer_", "global_", "flat_", "scratch_")) and not mn.startswith("buffer_wbl2") \
        and not mn.startswith("buffer_inv")


def is_store(mn):
    return is_vmem(mn) and ("_store" in mn or "_atomic" in mn)


def store_data(x):
    """VGPRs a store reads as data (buffer: operand 0; global / flat: operand 1)."""
    ops = _operands(x.ops)
    if x.mn.startswith("buffer_"):
        return _regs(ops[0]) if ops else set()
    return _regs(ops[1]) if len(ops) > 1 else set()


def valu_writes(x):
    if not x.mn.startswith("v_"):
        return set()
    ops = _operands(x.ops)
    if not ops:
        return set()
    w = _regs(ops[0])
    if "swap" in x.mn and len(ops) > 1:  # v_permlane16/32_swap, v_swap_b32 write both operands
        w |= _regs(ops[1])
    return w


def wide_store(x):
    return is_store(x.mn) and re.search(r"_dwordx[34]$|_format_xyzw?$|_b96$|_b128$", x.mn) is not None


def store_hazards(kern, ws=2, loads=False):
    """[(kernel, store addr, writer addr, writer, wait states in between)] for every store of more
    than 64 bits whose data VGPRs a VALU (or, with loads, a VMEM load) writes within ws wait states."""
    out = []
    for name, body in kern.items():
        by_addr = {x.addr: x.idx for x in body}
        for s in body:
            if not wide_store(s):
                continue
            data = store_data(s)
            seen = set()
            stack = [(j, 0) for j in successors(body, s.idx, by_addr)]
            while stack:
                j, w = stack.pop()
                if w >= ws or (j, w) in seen:
                    continue
                seen.add((j, w))
                x = body[j]
                hit = valu_writes(x)
                if loads and is_vmem(x.mn) and "_load" in x.mn:
                    hit = _regs(_operands(x.ops)[0]) if x.ops else set()
                if hit & data:
                    out.append((name, s.addr, x.addr, f"{x.mn} {x.ops}", w))
                    continue
                nw = w + (int(x.ops, 0) + 1 if x.mn == "s_nop" else 1)
                stack.extend((k, nw) for k in successors(body, j, by_addr))
    return out


def _vmcnt(x):
    if x.mn != "s_waitcnt":
        return None
    m = re.search(r"vmcnt\((\d+)\)", x.ops)
    return int(m.group(1)) if m else None


_SREG = re.compile(r"^(s\[\d+:\d+\]|s\d+|vcc|vcc_lo|vcc_hi|exec)$")


def _sregs(tok):
    m = re.match(r"^s\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"^s(\d+)$", tok)
    if m:
        return {int(m.group(1))}
    return {"vcc"} if tok.startswith("vcc") else {tok}


def _step_env(x, env):
    """Branch-condition constants after x: SGPRs set to -1 / 0 by s_mov, and vcc derived from them with
    exec (nonzero while the wave runs).  Anything else that writes an SGPR forgets it."""
    ops = _operands(x.ops)
    dst = ops[0] if ops else None
    env = dict(env)
    if x.mn in ("s_mov_b64", "s_mov_b32") and len(ops) == 2 and ops[1] in ("-1", "0"):
        env[dst] = int(ops[1])
        return env
    if x.mn in ("s_and_b64", "s_andn2_b64") and dst == "vcc" and len(ops) == 3 and ops[1] == "exec":
        v = env.get(ops[2])
        env.pop("vcc", None)
        if v is not None:
            keep = (v == -1) if x.mn == "s_and_b64" else (v == 0)
            env["vcc"] = "nz" if keep else 0
        return env
    if dst is not None and _SREG.match(dst) and (x.mn.startswith("s_") or x.mn.startswith(("v_readlane", "v_readfirstlane", "v_cmp"))):
        w = _sregs(dst)
        for key in [k for k in env if _sregs(k) & w]:
            env.pop(key, None)
    if x.mn.startswith("v_cmp") and "vcc" in x.ops:
        env.pop("vcc", None)
    return env


def _succ_env(body, i, by_addr, env):
    x = body[i]
    out = successors(body, i, by_addr)
    if x.mn in ("s_cbranch_vccz", "s_cbranch_vccnz") and "vcc" in env and len(out) == 2:
        taken = (env["vcc"] == 0) == (x.mn == "s_cbranch_vccz")
        out = [out[1]] if taken else [out[0]]
    return out


def flag_store_violations(kern, kernel_re, is_flag, mode, trace=False):
    """Row stores of kernels matching kernel_re that a flag store (is_flag(ins)) can publish before they
    have landed.  Forward from every row store S over every path (branches on vcc values known from
    s_mov constants are followed one way only): S is covered once a wait vmcnt(N) is reached with more
    than N memory operations issued after S.  A flag store reached while S is not covered is a
    violation in mode "all"; in mode "prev" only if another flag store was passed since S (S belongs
    to an entry whose ticket is still held back until then); in mode "prevN" (N = 1..9) only if N
    flag stores were passed since S (tickets published N + 1 entries late).  Returns ([(kernel, flag addr, reason)],
    flag stores in the checked kernels)."""
    bad, checked = [], 0
    allowed = int(mode[4:]) if mode.startswith("prev") and mode[4:] else 1
    for name, body in kern.items():
        if not re.search(kernel_re, name):
            continue
        by_addr = {x.addr: x.idx for x in body}
        checked += sum(1 for x in body if is_flag(x))
        starts = {0} | {by_addr[x.target] for x in body if x.target is not None} | \
            {x.idx + 1 for x in body if x.mn.startswith(("s_branch", "s_cbranch"))}
        for s in body:
            if not is_store(s.mn) or is_flag(s):
                continue
            # branch constants set earlier in S's basic block
            b0 = s.idx
            while b0 > 0 and b0 not in starts:
                b0 -= 1
            env0 = {}
            for y in body[b0:s.idx + 1]:
                env0 = _step_env(y, env0)
            envt0 = tuple(sorted(env0.items(), key=lambda kv: kv[0]))
            seen, parent = set(), {}
            stack = [(j, 0, 0, envt0) for j in _succ_env(body, s.idx, by_addr, env0)]
            found = None
            while stack and found is None:
                st = stack.pop()
                j, ops, flags, envt = st
                key = (j, ops, flags, envt)
                if key in seen:
                    continue
                seen.add(key)
                x = body[j]
                m = _vmcnt(x)
                if m is not None and ops >= m:
                    continue  # S has landed
                if is_flag(x):
                    if mode == "all" or flags >= allowed:
                        found = (name, x.addr, f"{x.mn} at {x.addr:#x} can publish row store {s.mn} at {s.addr:#x} "
                                               f"before it lands ({ops} later ops, waits insufficient)")
                        if trace:
                            path, cur = [], key
                            while cur is not None:
                                path.append(body[cur[0]])
                                cur = parent.get(cur)
                            found = found + ([f"{y.addr:#x} {y.mn} {y.ops}" for y in reversed(path)
                                              if is_vmem(y.mn) or y.mn == "s_waitcnt" or "branch" in y.mn
                                              or (y.mn.startswith("s_") and ("vcc" in y.ops or "s_mov" in y.mn))],)
                        break
                    flags = min(flags + 1, allowed)
                if is_vmem(x.mn):
                    ops = min(ops + 1, 64)
                env = _step_env(x, dict(envt))
                envt2 = tuple(sorted(env.items(), key=lambda kv: kv[0]))
                for k in _succ_env(body, j, by_addr, env):
                    nk = (k, ops, flags, envt2)
                    if trace and nk not in parent:
                        parent[nk] = key
                    stack.append(nk)
            if found:
                bad.append(found)
    return bad, checked


def progress_flag(x):
    """Progress / ticket / error words: one-dword agent-scope relaxed atomic stores (global_store_dword
    ... sc1); the sweeps' rows go through buffer instructions or wider global stores."""
    return x.mn == "global_store_dword" and " sc1" in f" {x.ops}"


def buffer_ticket(x):
    """k_det_sweep2's tickets: one-dword sc1 buffer stores (its f64 rows are dwordx2)."""
    return x.mn == "buffer_store_dword" and " sc1" in f" {x.ops}"


CHECKS = [
    # (kernel regex, mode, flag predicate): the systolic sweep publishes a cell only after ALL its
    # stores landed; the ticket sweeps publish update j-2's ticket at update j (j-1's stores may fly)
    (r"k_sweep_pair_sys", "all", progress_flag),
    (r"k_det_sweep2", "prev", buffer_ticket),
    (r"k_det_sweep_split", "prev", buffer_ticket),
    (r"k_online_sweepId", "prev", progress_flag),
    # kernels_online_sweep.hip: the single-item path publishes kSingle = 4 late (the general path 2,
    # which this allowance covers too)
    (r"k_online_f32", "prev3", progress_flag),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=DEFAULT_LIB)
    ap.add_argument("--ws", type=int, default=2)
    a = ap.parse_args()
    kern = kernels(a.lib)
    print(f"{len(kern)} kernels")
    for h in store_hazards(kern, a.ws):
        print("STORE-DATA HAZARD", h)
    for rx, mode, flag in CHECKS:
        bad, n = flag_store_violations(kern, rx, flag, mode)
        print(f"{rx}: {n} flag stores checked, {len(bad)} violations")
        for b in bad[:10]:
            print("  ", b)


if __name__ == "__main__":
    main()


def explain(kern, name, s_addr, f_addr):
    """The path from row store s_addr to flag store f_addr with the fewest memory operations
    (debugging aid): its memory operations, waits and branches."""
    import heapq
    body = kern[name]
    by_addr = {x.addr: x.idx for x in body}
    src, dst = by_addr[s_addr], by_addr[f_addr]
    dist, prev, pq = {src: 0}, {}, [(0, src)]
    while pq:
        d, i = heapq.heappop(pq)
        if i == dst:
            break
        if d > dist.get(i, 1 << 30):
            continue
        for j in successors(body, i, by_addr):
            nd = d + (1 if is_vmem(body[j].mn) else 0)
            if nd < dist.get(j, 1 << 30):
                dist[j], prev[j] = nd, i
                heapq.heappush(pq, (nd, j))
    path = [dst]
    while path[-1] != src:
        path.append(prev[path[-1]])
    lines = []
    for i in reversed(path):
        x = body[i]
        if is_vmem(x.mn) or x.mn == "s_waitcnt" or "branch" in x.mn or (x.mn.startswith("s_") and "vcc" in x.ops):
            lines.append(f"{x.addr:#x} {x.mn} {x.ops}" + (f" -> {x.target:#x}" if x.target else ""))
    return lines
