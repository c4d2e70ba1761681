"""tools/vmcnt_check.py -- check the zstd decoder's counted-wait invariant on the BUILT code object.

The per-lane zstd decode kernels (`lzh_zstd_seq_kernel`, `lzh_zstd_huf_kernel`, `lzh_zstd_huf8_kernel`,
lzbench_amd/csrc/decode_hip.hip) fill LDS by LDS-DMA (`global_load_lds_dword`) at a uniform point and
read those rows after the NEXT uniform point's `s_waitcnt vmcnt(16)`.  Nothing but the issuing wave's
vmcnt orders a ds_read behind a pending LDS-DMA (MI355X_MICROARCH.md, "Two waves per SIMD", item 7),
and vector-memory operations complete in issue order, so that wait covers the fills only if at least
16 vector-memory operations were issued after the last fill on EVERY path from it to the wait (the
kernels store exactly one record / byte per step, 16 steps per interval, a dummy one when a lane has
none).  Fewer -- a per-step store that the compiler turns into a branch skipped when no lane stores,
or an interval the compiler shortens -- and the wait lets the fills still be in flight: the steps then
read stale LDS bytes (wrong output, no fault).  More operations only make the wait stricter.

This is a forward data-flow over the disassembly's control-flow graph: the state at an instruction is
the MINIMUM, over all paths reaching it, of the vector-memory operations issued since the most recent
LDS-DMA fill (infinity: no fill pending).  A fill sets 0, any other vector-memory instruction adds 1, a
`s_waitcnt vmcnt(k)` reached with state >= k retires every fill (infinity).  Every `s_waitcnt vmcnt(16)`
must be reached with state >= 16.

usage: python tools/vmcnt_check.py [object.o]   (default build/obj/decode_hip.o)
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
KERNELS = ("lzh_zstd_seq_kernel", "lzh_zstd_huf_kernel", "lzh_zstd_huf8_kernel")
POINT_WAIT = 16
INF = 1 << 30

_ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")
_TARGET = re.compile(r"<([A-Za-z0-9_.$]+)\+0x([0-9a-f]+)>")
_VMCNT = re.compile(r"vmcnt\((\d+)\)")


def disassemble(obj: str) -> str:
    """Disassembly (llvm-objdump, gfx950) of the device code object inside a hipcc -c object."""
    with tempfile.TemporaryDirectory() as td:
        fat, co = os.path.join(td, "fat.bin"), os.path.join(td, "dev.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                              capture_output=True, text=True).stdout


def kernel_listing(dis: str, name: str) -> list[tuple[int, str]]:
    """[(address, instruction text)] of one function of the disassembly."""
    out, on = [], False
    for line in dis.splitlines():
        if line.endswith(">:") and "<" in line:
            on = line.split("<", 1)[1][:-2] == name
            continue
        if not on or not line.startswith("\t"):
            continue
        m = _ADDR.search(line)
        if m:
            out.append((int(m.group(1), 16), line.split("//")[0].strip()))
    if not out:
        raise ValueError(f"{name}: not in the disassembly")
    return out


def is_vmem(ins: str) -> bool:
    op = ins.split()[0]
    return op.startswith(("global_", "buffer_", "flat_", "scratch_", "tbuffer_"))


def is_fill(ins: str) -> bool:
    op = ins.split()[0]
    return op.startswith("global_load_lds") or (op.startswith("buffer_load") and " lds" in f" {ins}")


_SREG = re.compile(r"^s(\d+)$")
# scalar instructions that leave SCC alone (every other s_ instruction may write it)
_KEEPS_SCC = ("s_mov_b32", "s_mov_b64", "s_movk_i32", "s_waitcnt", "s_nop", "s_setprio", "s_sleep", "s_barrier",
              "s_getreg_b32", "s_branch", "s_cbranch", "s_memtime", "s_memrealtime", "s_sethalt", "s_load",
              "s_buffer_load", "s_dcache_inv", "s_inst_prefetch", "s_setreg", "s_cselect")


def _imm(tok: str):
    try:
        return int(tok, 0)
    except ValueError:
        return None


def _writes_exec(ins: str) -> bool:
    toks = ins.replace(",", " ").split()
    return "saveexec" in toks[0] or (len(toks) > 1 and toks[0].startswith("s_") and toks[1] == "exec")


def _succ(lst, name, base):
    """Successor lists of the listing (instruction indices), with the branch kind of each conditional
    branch.  Branches on exec: the exec-zero edge (taken for s_cbranch_execz, fall-through for
    s_cbranch_execnz) is kept only when exec was narrowed in the branch's own basic block (the
    `if` of a lane-divergent region: its body, a store included, is skipped when no lane enters).
    Without such a write the branch is the structurizer's flow block at the exit of a wave-uniform
    loop (seen on `if (!ballot(..)) break;`), where exec is the whole wave and is never zero."""
    index = {a: i for i, (a, _) in enumerate(lst)}
    targets = set()
    for a, ins in lst:
        op = ins.split()[0]
        if op == "s_branch" or op.startswith("s_cbranch"):
            imm = int(ins.split()[1])
            targets.add(a + 4 + 4 * (imm - (1 << 16) if imm >= 1 << 15 else imm))
    succ = []
    for i, (a, ins) in enumerate(lst):
        op = ins.split()[0]
        nxt = [i + 1] if i + 1 < len(lst) else []
        if op.startswith(("s_setpc", "s_swappc", "s_call")):
            raise ValueError(f"{name}: {op} at {a:#x}: calls are not modelled")
        if op in ("s_endpgm", "s_trap"):
            succ.append(([], None))
            continue
        if op == "s_branch" or op.startswith("s_cbranch"):
            imm = int(ins.split()[1])
            imm = imm - (1 << 16) if imm >= 1 << 15 else imm
            tgt = a + 4 + 4 * imm
            if tgt not in index:
                raise ValueError(f"{name}: branch at {a:#x} to {tgt:#x} outside the kernel")
            if op == "s_branch":
                succ.append(([index[tgt]], None))
                continue
            if op in ("s_cbranch_execz", "s_cbranch_execnz"):
                narrowed = False
                for j in range(i - 1, -1, -1):
                    pj = lst[j][1].split()[0]
                    if pj == "s_branch" or pj.startswith("s_cbranch") or pj == "s_endpgm":
                        break
                    if _writes_exec(lst[j][1]):
                        narrowed = True
                        break
                    if lst[j][0] in targets:
                        break
                if not narrowed:   # only the exec-nonzero edge
                    succ.append(([index[tgt]] if op == "s_cbranch_execnz" else nxt, None))
                    continue
            succ.append(([index[tgt]] + nxt, op))   # (taken, fall-through)
            continue
        succ.append((nxt, None))
    return succ


def _step(ins, consts, scc):
    """Scalar constant tracking through one instruction: (consts, scc) after it.  Tracks SGPRs set
    from an immediate and stepped by an immediate (loop counters), and SCC from a compare of one."""
    toks = ins.replace(",", " ").split()
    op = toks[0]
    args = toks[1:]
    dst = _SREG.match(args[0]) if args else None
    c = dict(consts)
    if op in ("s_mov_b32", "s_movk_i32") and dst:
        v = _imm(args[1])
        c.pop(args[0], None)
        if v is not None and -4096 <= v <= 4096:
            c[args[0]] = v
        return c, scc
    if op in ("s_add_i32", "s_sub_i32", "s_add_u32", "s_sub_u32") and dst and len(args) == 3:
        v = c.get(args[1]) if args[1] == args[0] else None
        k = _imm(args[2])
        c.pop(args[0], None)
        if v is not None and k is not None:
            c[args[0]] = v + k if op.startswith("s_add") else v - k
        return c, None
    if op == "s_addk_i32" and dst:
        v, k = c.get(args[0]), _imm(args[1])
        c.pop(args[0], None)
        if v is not None and k is not None:
            c[args[0]] = v + k
        return c, None
    if op.startswith(("s_cmp_", "s_cmpk_")):
        a, b = args[0], args[1]
        va = c.get(a) if _SREG.match(a) else _imm(a)
        vb = c.get(b) if _SREG.match(b) else _imm(b)
        if va is None or vb is None:
            return c, None
        rel = op.split("_")[-2]
        res = {"eq": va == vb, "lg": va != vb, "gt": va > vb, "ge": va >= vb, "lt": va < vb, "le": va <= vb}.get(rel)
        return c, res
    # any other writer of a tracked SGPR forgets it (scalar and vector-to-scalar forms alike)
    for a in args[:1]:
        for r in re.findall(r"s\[(\d+):(\d+)\]", a):
            for k in range(int(r[0]), int(r[1]) + 1):
                c.pop(f"s{k}", None)
        if dst:
            c.pop(a, None)
    if op.startswith("s_") and not op.startswith(_KEEPS_SCC):
        scc = None
    return c, scc


def check_listing(lst: list[tuple[int, str]], name: str, base: int | None = None) -> list[str]:
    """Problems found in one kernel's listing (empty: the invariant holds on every path).

    Path exploration from every LDS-DMA fill: the state is (instruction, vector-memory operations since
    the fill, known scalar constants, SCC).  SCC-conditioned branches whose SCC is known (a loop counter
    set from an immediate, stepped by an immediate, compared with one) take only their feasible edge, so
    a counted step loop is walked its real number of times.  A path ends at s_endpgm, at any
    s_waitcnt vmcnt(k) with k <= the count (the fill retired), or at a count of 16 or more (safe)."""
    if base is None:
        base = lst[0][0]
    succ = _succ(lst, name, base)
    problems = []
    fills = [i for i, (_, ins) in enumerate(lst) if is_fill(ins)]
    seen = set()
    for f0 in fills:
        stack = [(f0 + 1, 0, (), None)]
        while stack:
            i, cnt, cst, scc = stack.pop()
            key = (i, cnt, cst, scc)
            if key in seen or i >= len(lst):
                continue
            seen.add(key)
            a, ins = lst[i]
            m = _VMCNT.search(ins) if ins.startswith("s_waitcnt") else None
            if m:
                k = int(m.group(1))
                if k == POINT_WAIT and cnt < POINT_WAIT:
                    problems.append(f"{name}+{a - base:#x}: {ins} reachable with only {cnt} vector-memory "
                                    f"operations after the LDS-DMA fill at +{lst[f0][0] - base:#x} (need >= {POINT_WAIT})")
                    continue
                if cnt >= k:
                    continue                     # the fill is retired on this path
            if is_fill(ins):
                continue                         # (a later fill: explored from there)
            if is_vmem(ins):
                cnt += 1
                if cnt >= POINT_WAIT:
                    continue
            c, s2 = _step(ins, dict(cst), scc)
            nx, cond = succ[i]
            if cond in ("s_cbranch_scc1", "s_cbranch_scc0") and s2 is not None and len(nx) == 2:
                taken = s2 if cond == "s_cbranch_scc1" else not s2
                nx = [nx[0]] if taken else [nx[1]]
            ct = tuple(sorted(c.items()))
            for j in nx:
                stack.append((j, cnt, ct, s2))
        if len(problems) > 20:
            break
    points = sum(1 for _, ins in lst if ins.startswith("s_waitcnt") and f"vmcnt({POINT_WAIT})" in ins)
    if points == 0:
        problems.append(f"{name}: no s_waitcnt vmcnt({POINT_WAIT}) uniform point found")
    if not fills:
        problems.append(f"{name}: no LDS-DMA fill found")
    return sorted(set(problems))


def check_object(obj: str) -> dict[str, list[str]]:
    dis = disassemble(obj)
    return {k: check_listing(kernel_listing(dis, k), k) for k in KERNELS}


if __name__ == "__main__":
    obj = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "build", "obj", "decode_hip.o")
    bad = 0
    for k, probs in check_object(obj).items():
        print(f"{k}: {'ok' if not probs else 'FAIL'}")
        for p in probs:
            print("   ", p)
        bad += len(probs)
    sys.exit(1 if bad else 0)
