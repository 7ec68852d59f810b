#!/usr/bin/env python3
"""Build-time ISA hazard check of librnsntt's gfx950 code objects.

hipcc's hazard recognizer pads the MFMA hazards of the instructions it
generates, but not of inline asm (it schedules an asm statement as one opaque
instruction), and it never counts an asm load's completion.  This scans the
disassembly of every kernel in the given objects and reports, per kernel:

  M1  a VGPR written by an MFMA (D) read or written by a later non-chained
      instruction fewer than W_D wait states after that MFMA issued;
  M2  a VGPR an MFMA reads (A, B or C) written by a later instruction fewer
      than W_SRC wait states after it issued (the MFMA is still in flight);
  M3  an MFMA whose D overlaps its A or B operand (partly or wholly);
  M4  an MFMA operand written by a VALU / LDS / VMEM instruction fewer than
      W_IN wait states before the MFMA;
  L1  a VGPR that a DS / VMEM / scratch load writes, read or written before
      the s_waitcnt that retires that load (the loads of inline asm are not
      in hipcc's bookkeeping; a compiler copy of such a register before the
      wait reads stale data);
  S1  a VGPR holding the data of a VMEM store of more than 64 bits written
      by a VALU instruction fewer than W_ST wait states after the store
      issued.  The store reads
      its data after issue; hipcc pads this hazard only for stores without
      an SGPR soffset (LLVM's createsVALUHazard), but on gfx950 a buffer
      store with an SGPR soffset lost single lanes of its data to a
      `v_mov_b32` into the data register 0-1 states later (r05: k_mf_tensor's
      scratch-slot words, profiles/r05/ab_mf_ntt_split_load.txt).

Wait states: one per instruction, N+1 for `s_nop N` (the ISA's counting,
and LLVM's).  v_mfma_i32_16x16x64_i8 is a 4-pass XDL op on gfx950 (16
cycles: the cycles of bf16 16x16x32, MI355X_MICROARCH.md "Matrix cores");
hipcc's own window for an XDL D -> VALU read at 4 passes is 8 states
(passes + 3, + 1 on gfx950), visible in every tile it emits.  The rule this
repo applies ("MFMA hazards") is stricter and uniform: nothing
touches any register an MFMA reads or writes until W_D = 8 states after the
LAST MFMA of a tile has issued, an MFMA's D never overlaps its A/B, and an
MFMA operand written by VALU / memory is 2+ states old at issue.

  X1  a kernel with loops whose loop-carried states (in-flight MFMAs, wide
      stores, un-waited loads) do not reach a fixpoint: back edges are
      followed, so a loop-carried hazard is checked like a straight-line one.

Exit status 1 if any finding; `--allow KERNEL_SUBSTR` skips kernels.
Usage: isa_check.py OBJ.o [OBJ.o ...] [--verbose]
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
W_D = 8     # MFMA D -> any access (4-pass XDL on gfx950: passes + 4)
W_SRC = 8   # MFMA A/B/C -> overwrite (in flight until its D is written)
W_IN = 2    # VALU/memory write -> MFMA operand read
W_ST = 2    # VMEM store (> 64-bit data) -> overwrite of its data VGPRs

REG = re.compile(r"^([vas])(?:(\d+)|\[(\d+):(\d+)\])$")


def regs(tok: str):
    """('v', {5,6}) for v[5:6]; None for non-register operands."""
    m = REG.match(tok)
    if not m:
        return None
    kind = m.group(1)
    if m.group(2) is not None:
        lo = hi = int(m.group(2))
    else:
        lo, hi = int(m.group(3)), int(m.group(4))
    return kind, set(range(lo, hi + 1))


def vset(toks):
    out = set()
    for t in toks:
        r = regs(t)
        if r and r[0] in "va":
            out |= {(r[0], i) for i in r[1]}
    return out


def split_ops(s: str):
    s = s.split("//")[0].strip()
    parts = s.split(None, 1)
    mn = parts[0]
    rest = parts[1] if len(parts) > 1 else ""
    ops = [o.strip() for o in rest.split(",")] if rest else []
    # strip modifiers ("0 offen offset:16", "off offset:12")
    clean = []
    for o in ops:
        clean.append(o.split()[0] if o else o)
    return mn, clean, rest


def defs_uses(mn: str, ops):
    """VGPR/AGPR defs and uses of one instruction."""
    if mn.startswith("s_") or not ops:
        return set(), set()
    if mn.startswith("v_mfma"):
        return vset(ops[:1]), vset(ops[1:])
    if mn.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
        return set(), vset(ops[1:])
    if mn.startswith(("v_permlane16_swap", "v_permlane32_swap")):
        s = vset(ops[:2])
        return s, s
    if mn.startswith("v_writelane"):
        s = vset(ops[:1])
        return s, s | vset(ops[1:])
    if mn.startswith(("global_load_lds", "buffer_load_lds")) or (mn.startswith("buffer_load") and " lds" in " ".join(ops)):
        return set(), vset(ops)  # LDS DMA: the first operand is the address
    if mn.startswith(("ds_read", "buffer_load", "global_load", "scratch_load", "flat_load")):
        return vset(ops[:1]), vset(ops[1:])
    if mn.startswith(("ds_write", "buffer_store", "global_store", "scratch_store", "flat_store")):
        return set(), vset(ops)
    if mn.startswith("v_"):
        return vset(ops[:1]), vset(ops[1:])
    if mn.startswith("ds_"):  # ds_swizzle, ds_bpermute, ds_add_rtn...
        return vset(ops[:1]), vset(ops[1:])
    return set(), vset(ops)


def wait_states(mn: str, ops):
    if mn == "s_nop":
        return int(ops[0], 0) + 1
    return 1


def load_kind(mn: str):
    if mn.startswith("ds_read") or (mn.startswith("ds_") and "rtn" in mn) or mn.startswith(("ds_swizzle", "ds_bpermute", "ds_permute")):
        return "lgkm"
    if mn.startswith(("buffer_load", "global_load", "scratch_load", "flat_load")):
        return "vm"
    return None


def store_kind(mn: str):
    if mn.startswith(("buffer_store", "global_store", "scratch_store", "flat_store")):
        return "vm"
    if mn.startswith("ds_write"):
        return "lgkm"
    return None


WAITCNT = re.compile(r"(vmcnt|lgkmcnt|expcnt)\((\d+)\)")


def disassemble(obj: str, tmp: str):
    fat = os.path.join(tmp, "fat.bin")
    co = os.path.join(tmp, "dev.co")
    secs = subprocess.run([f"{LLVM}/llvm-readelf", "-S", obj], check=True, capture_output=True, text=True).stdout
    if ".hip_fatbin" not in secs:
        return ""  # host code only
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(tmp, "x.o")],
                   check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True, capture_output=True,
                         text=True).stdout
    return out


def kernels(dis: str):
    cur, body, faddr = None, [], 0
    for line in dis.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            if cur:
                yield cur, faddr, body
            cur, body, faddr = m.group(2), [], int(m.group(1), 16)
            continue
        if cur and line.startswith("\t"):
            txt = line.strip()
            addr = None
            am = re.search(r"//\s*([0-9A-F]+):", txt)
            if am:
                addr = int(am.group(1), 16)
            body.append((addr, txt))
    if cur:
        yield cur, faddr, body


TARGET = re.compile(r"<[^>+]+\+0x([0-9a-f]+)>")
BRANCHES = ("s_branch", "s_cbranch_")


class State:
    """What is in flight at one point of the code: MFMAs (issue counter,
    D, operands), wide stores still reading their data, un-waited loads and
    stores, and the last VALU write of each register.  Counters are
    wait-state counts along the path.  Un-waited memory ops are kept as
    op -> depth, the number of ops of the same counter issued after it
    (`s_waitcnt vmcnt(n)` retires exactly the ops of depth >= n: returns are
    in order); where paths join, an op keeps its smallest depth (pending on
    any path means pending), so the state is path-insensitive and finite."""

    def __init__(self):
        self.mfmas = []        # dict(end, dst, srcs, text)
        self.stores = []       # dict(end, data, text): wide VMEM stores still reading their data
        self.pend = {}         # (kind, regs, text) -> depth
        self.last_write = {}   # reg -> counter after the write

    def copy(self):
        t = State()
        t.mfmas = [dict(f) for f in self.mfmas]
        t.stores = [dict(f) for f in self.stores]
        t.pend = dict(self.pend)
        t.last_write = dict(self.last_write)
        return t

    def shifted(self, delta):
        t = self.copy()
        for f in t.mfmas + t.stores:
            f["end"] += delta
        t.last_write = {r: v + delta for r, v in t.last_write.items()}
        return t

    def merge(self, o):
        seen = {(f["text"], f["end"]) for f in self.mfmas}
        self.mfmas += [f for f in o.mfmas if (f["text"], f["end"]) not in seen]
        seen = {(f["text"], f["end"]) for f in self.stores}
        self.stores += [f for f in o.stores if (f["text"], f["end"]) not in seen]
        for k, dpt in o.pend.items():
            self.pend[k] = min(dpt, self.pend.get(k, dpt))
        for r, v in o.last_write.items():
            self.last_write[r] = max(v, self.last_write.get(r, -10**9))


AGE_CAP = 64  # wait states after which nothing in State can still matter (W_D, W_SRC, W_IN, W_ST < 64)
MAX_ITERS = 16
VM_CAP = 64    # outstanding ops of one counter kept per path (vmcnt is a 6-bit counter)


def _normalize(st: State, at: int) -> State:
    """The state at a back-edge branch, ages relative to the branch (ends
    made <= 0), with everything too old to matter dropped: a finite form, so
    the loop iteration below reaches a fixpoint."""
    t = st.shifted(-at)
    t.mfmas = [f for f in t.mfmas if -f["end"] < AGE_CAP]
    t.stores = [f for f in t.stores if -f["end"] < W_ST]
    t.last_write = {r: v for r, v in t.last_write.items() if -v < W_IN}
    return t


def _signature(st: State):
    return (frozenset((f["text"], f["end"]) for f in st.mfmas),
            frozenset((f["text"], f["end"]) for f in st.stores),
            frozenset(st.pend.items()),
            frozenset(st.last_write.items()))


def _scan(body, func_addr, back_in):
    """One pass over the kernel in address order.  Forward branches carry
    their state to the target (merged with the fall-through path); back
    edges carry theirs (normalized) into the next pass through `back_in`.
    Returns the findings and the back-edge states this pass produced."""
    findings = []
    back_out = {}
    st = State()
    pending = {}  # target addr -> list of (State, counter at the branch)
    since = 0
    live = True   # the fall-through path reaches this instruction
    for idx, (addr, txt) in enumerate(body):
        arrivals = list(pending.pop(addr, [])) if addr is not None else []
        if addr is not None and addr in back_in:
            arrivals.append((back_in[addr], 0))  # normalized: ages relative to its branch
        if arrivals:
            base = st if live else None
            for s_b, c_b in arrivals:
                # the taken branch counts as its one wait state (already in
                # c_b), nothing more: conservative
                moved = s_b.shifted(since - c_b)
                if base is None:
                    base = moved
                else:
                    base.merge(moved)
            st = base
            live = True
        if not live:
            st = State()  # reached by no path in this scan
            live = True
        mn, ops, rest = split_ops(txt)
        d, u = defs_uses(mn, ops)
        ws = wait_states(mn, ops)
        # ---- L1: accesses to registers of loads not yet waited for
        if mn == "s_waitcnt":
            cnts = {k: int(v) for k, v in WAITCNT.findall(rest)}
            for kind in ("vm", "lgkm"):
                key = "vmcnt" if kind == "vm" else "lgkmcnt"
                if key not in cnts:
                    continue
                n = cnts[key]
                st.pend = {o: dp for o, dp in st.pend.items() if o[0] != kind or dp < n}
        elif not mn.startswith("s_"):
            touched = d | u
            lk0 = load_kind(mn)
            for o in st.pend:
                if lk0 == o[0] and not (o[1] & u):
                    continue  # a later load of the same counter: returns in order, lands last
                if o[1] and (o[1] & touched):
                    findings.append(("L1", idx, f"{txt}  touches {sorted(o[1] & touched)[:4]} of un-waited load `{o[2]}`"))
        lk = load_kind(mn)
        sk = store_kind(mn)
        op = None
        if mn.startswith("s_load") or mn.startswith("s_buffer_load"):
            op = ("lgkm", frozenset(), f"{idx}: " + txt.split("//")[0].strip())
        elif lk:
            op = (lk, frozenset(d), f"{idx}: " + txt.split("//")[0].strip())
        elif sk:
            op = (sk, frozenset(), f"{idx}: " + txt.split("//")[0].strip())
        if op:
            # one more op behind every pending op of its counter; beyond
            # VM_CAP the counter cannot hold them: those have retired
            st.pend = {o: dp + (o[0] == op[0]) for o, dp in st.pend.items()
                       if dp + (o[0] == op[0]) < VM_CAP}
            st.pend[op] = 0
        # ---- MFMA rules
        is_mf = mn.startswith("v_mfma")
        if is_mf:
            a, b, c = vset(ops[1:2]), vset(ops[2:3]), vset(ops[3:4])
            if vset(ops[:1]) & (a | b):
                findings.append(("M3", idx, f"{txt}  D overlaps A/B"))
            for r in a | b | c:
                if r in st.last_write and since - st.last_write[r] < W_IN:
                    findings.append(("M4", idx, f"{txt}  operand {r} written {since - st.last_write[r]} states before"))
        for f in st.mfmas:
            dist = since - f["end"]  # wait states between its issue and this instruction
            if dist >= max(W_D, W_SRC):
                continue
            if is_mf:
                cset = vset(ops[3:4])
                if f["dst"] & vset(ops[1:3]) and dist < W_D:
                    findings.append(("M1", idx, f"{txt}  reads D of `{f['text']}` as A/B after {dist}"))
                if f["dst"] & cset and cset != f["dst"] and dist < W_D:
                    findings.append(("M1", idx, f"{txt}  partial C overlap with D of `{f['text']}`"))
                if (vset(ops[:1]) & f["srcs"]) and dist < W_SRC and vset(ops[:1]) != f["dst"]:
                    findings.append(("M2", idx, f"{txt}  writes an operand of in-flight `{f['text']}` after {dist}"))
                continue
            if mn.startswith("s_"):
                continue
            if (f["dst"] & (d | u)) and dist < W_D:
                findings.append(("M1", idx, f"{txt}  touches D {sorted(f['dst'] & (d | u))[:4]} of `{f['text']}` after {dist} states"))
            if (f["srcs"] & d) and dist < W_SRC:
                findings.append(("M2", idx, f"{txt}  overwrites operand {sorted(f['srcs'] & d)[:4]} of `{f['text']}` after {dist} states"))
        # ---- S1: data registers of a wide store still being read
        if mn.startswith("v_"):  # VALU writers (a load's data returns far later)
            for f in st.stores:
                if (f["data"] & d) and since - f["end"] < W_ST:
                    findings.append(("S1", idx, f"{txt}  overwrites data {sorted(f['data'] & d)[:4]} of `{f['text']}` "
                                                f"after {since - f['end']} states"))
        since += ws
        if sk == "vm":
            data = vset(ops[:1]) if mn.startswith("buffer_store") else vset(ops[1:2])
            if len(data) > 2:
                st.stores.append({"end": since, "data": data, "text": txt.split("//")[0].strip()})
        st.stores = [f for f in st.stores if since - f["end"] < W_ST]
        if is_mf:
            st.mfmas.append({"end": since, "dst": vset(ops[:1]), "srcs": vset(ops[1:]), "text": txt.split("//")[0].strip()})
        st.mfmas = [f for f in st.mfmas if since - f["end"] < AGE_CAP]
        if mn.startswith("v_") and not is_mf:
            for r in d:
                st.last_write[r] = since
        # ---- control flow
        if mn.startswith(BRANCHES):
            m = TARGET.search(txt)
            if m:
                tgt = func_addr + int(m.group(1), 16)
                if addr is None or tgt > addr:
                    pending.setdefault(tgt, []).append((st.copy(), since))
                else:  # back edge: into the next pass, at the loop head
                    nb = _normalize(st, since)
                    if tgt in back_out:
                        back_out[tgt].merge(nb)
                    else:
                        back_out[tgt] = nb
            if mn == "s_branch":
                live = False
        elif mn in ("s_setpc_b64", "s_endpgm"):
            live = False
    return findings, back_out


def check_kernel(body, func_addr, verbose=False):
    """Every path of the kernel, loops included: passes over the code in
    address order, each feeding the states its back edges carry to their
    loop heads into the next, until those states stop changing (a fixpoint:
    every loop-carried hazard -- an MFMA, a wide store or a load still in
    flight across the back edge -- has then reached the loop body).  The
    findings of every pass are reported; a kernel whose loop states do not
    converge within MAX_ITERS passes is itself a finding (X1), so a looping
    kernel is never passed unchecked."""
    back_in = {}
    found = {}
    for _ in range(MAX_ITERS):
        fs, back_out = _scan(body, func_addr, back_in)
        for f in fs:
            found.setdefault((f[0], f[1], f[2]), f)
        merged = {}
        for tgt in set(back_in) | set(back_out):
            m = back_in[tgt].copy() if tgt in back_in else None
            if tgt in back_out:
                if m is None:
                    m = back_out[tgt].copy()
                else:
                    m.merge(back_out[tgt])
            merged[tgt] = m
        if {t: _signature(v) for t, v in merged.items()} == {t: _signature(v) for t, v in back_in.items()}:
            break
        back_in = merged
    else:
        found[("X1", 0, "loop states did not converge")] = (
            "X1", 0, f"loop-carried states did not converge in {MAX_ITERS} passes")
    return sorted(found.values(), key=lambda f: (f[1], f[0]))


def main(argv):
    verbose = "--verbose" in argv
    allow = []
    objs = []
    it = iter(argv)
    for a in it:
        if a == "--verbose":
            continue
        if a == "--allow":
            allow.append(next(it))
            continue
        objs.append(a)
    total = 0
    with tempfile.TemporaryDirectory() as tmp:
        for obj in objs:
            dis = disassemble(obj, tmp)
            for name, faddr, body in kernels(dis):
                if any(s in name for s in allow):
                    continue
                fs = check_kernel(body, faddr, verbose)
                n_mf = sum(1 for _, t in body if t.startswith("v_mfma"))
                kinds = {}
                for k, _, _ in fs:
                    kinds[k] = kinds.get(k, 0) + 1
                if fs or verbose:
                    print(f"{os.path.basename(obj)} {name[:70]}: {len(body)} instrs, {n_mf} MFMA, findings {kinds}")
                for k, i, msg in fs[: (10**9 if verbose else 12)]:
                    print(f"  [{k}] #{i}: {msg}")
                total += len(fs)
    print(f"isa_check: {total} finding(s)")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
