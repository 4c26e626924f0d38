"""Build-time check of the shipped gfx950 code object: no instruction touches a register whose load
is still in flight.

Why.  k_mm_wave loads its MFMA operands with inline-asm `buffer_load_dwordx4`
and waits with counted `s_waitcnt vmcnt(N)`; k_mm_ring reads LDS with inline-asm `ds_read_b128`.
The compiler sees an asm output as defined at the asm statement, so nothing stops it from copying
or reusing that register before the wait -- a register-allocation change away from wrong results
(the round-5 bf16x3 probe hit exactly that).  The compiler's own loads are always
covered by the waits it inserts; the inline-asm ones are not.  So after every build this module
disassembles the gfx950 code object inside libgta.so (llvm-objdump --offloading, then -d) and runs
a data-flow pass over every kernel's control-flow graph:

  * state = the in-flight memory operations in issue order, per counter: vmcnt (buffer_ / global_ /
    flat_ / scratch_ operations, loads and stores alike on gfx9) and lgkmcnt (ds_ operations, scalar
    memory loads, flat operations, s_sendmsg), each with the registers it will write;
  * `s_waitcnt vmcnt(N)` retires all but the N newest vm operations (they return in order);
    `lgkmcnt(N)` does the same for LDS operations, but scalar loads return out of order, so with one
    in flight only lgkmcnt(0) retires anything;
  * at a control-flow join the states are merged position by position from the newest end (a wait
    keeps the newest N), taking the union of registers -- conservative for every path;
  * a hazard is any instruction that reads or writes a register an in-flight load will write.

`_build.build()` fails on any hazard (tests/test_abi.py runs the check on the built library in the
CPU suite).  Run by hand: python -m gta_graph_tensor_acclelrator_for_general_gnn_amd.asmcheck [libgta.so]
"""
import glob
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM_BIN = "/opt/rocm/lib/llvm/bin"
QCAP = 64  # a counter holds at most 63 operations; older entries are treated as returned

_FUNC = re.compile(r"^([0-9a-f]+) <([^>]+)>:\s*$")
_INSN = re.compile(r"^\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-F]+):[^<]*(?:<([^>+]+)(?:\+0x([0-9a-f]+))?>)?\s*$")
_VREG = re.compile(r"\b([va])(?:(\d+)\b|\[(\d+):(\d+)\])")
_SREG = re.compile(r"\bs(?:(\d+)\b|\[(\d+):(\d+)\])")
_WAIT = re.compile(r"(vmcnt|lgkmcnt)\((\d+)\)")


def objdump():
    for c in (os.path.join(LLVM_BIN, "llvm-objdump"), shutil.which("llvm-objdump")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("llvm-objdump not found")


def disassemble(so_path, arch="gfx950"):
    """Disassembly text of the `arch` code object embedded in so_path."""
    tmp = tempfile.mkdtemp(prefix="gta_asmcheck_")
    try:
        lib = os.path.join(tmp, "lib.so")
        shutil.copyfile(so_path, lib)
        subprocess.run([objdump(), "--offloading", lib], check=True, cwd=tmp, capture_output=True)
        cos = [p for p in glob.glob(os.path.join(tmp, "lib.so.*")) if p.endswith(arch)]
        if len(cos) != 1:
            raise RuntimeError(f"expected one {arch} code object in {so_path}, found {cos}")
        r = subprocess.run([objdump(), "-d", f"--mcpu={arch}", cos[0]], check=True, capture_output=True, text=True)
        return r.stdout
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def _regs(text, pattern):
    out = set()
    for m in pattern.finditer(text):
        g = m.groups()
        if len(g) == 4:  # v / a registers: keep the file apart
            kind, one, lo, hi = g
            rng = [int(one)] if one is not None else range(int(lo), int(hi) + 1)
            out.update(f"{kind}{r}" for r in rng)
        else:
            one, lo, hi = g
            rng = [int(one)] if one is not None else range(int(lo), int(hi) + 1)
            out.update(f"s{r}" for r in rng)
    return out


def parse(text):
    """{kernel name: [(addr, mnemonic, operands, branch target addr or None)]}."""
    funcs, cur, base = {}, None, 0
    for line in text.splitlines():
        m = _FUNC.match(line)
        if m:
            base = int(m.group(1), 16)
            cur = funcs.setdefault(m.group(2), [])
            continue
        if cur is None:
            continue
        m = _INSN.match(line)
        if not m:
            continue
        mn, ops, addr, tsym, toff = m.groups()
        tgt = None
        if (mn.startswith("s_branch") or mn.startswith("s_cbranch")) and tsym is not None:
            tgt = base + (int(toff, 16) if toff else 0)
        cur.append((int(addr, 16), mn, ops, tgt))
    return funcs


def classify(mn, ops):
    """(counts on vmcnt, counts on lgkmcnt, scalar memory, registers the operation will write late)."""
    vm = mn.startswith(("buffer_", "global_", "scratch_", "flat_"))
    lgkm = mn.startswith(("ds_", "s_load", "s_buffer_load", "s_scratch_load", "flat_", "s_sendmsg", "s_memtime",
                          "s_memrealtime", "s_dcache", "s_atc_probe"))
    smem = mn.startswith(("s_load", "s_buffer_load", "s_scratch_load", "s_memtime", "s_memrealtime"))
    dest = set()
    first = ops.split(",")[0] if ops else ""
    if vm or lgkm:
        returns = ("_load" in mn and "_load_lds" not in mn and not ops.rstrip().endswith(" lds")) or \
                  mn.startswith("ds_read") or ("_atomic" in mn and re.search(r"\b(glc|sc0)\b", ops)) or \
                  (mn.startswith("ds_") and "_rtn" in mn) or mn in ("s_memtime", "s_memrealtime")
        if returns:
            dest = _regs(first, _SREG) if smem else _regs(first, _VREG)
    return vm, lgkm, smem, dest


def _join(a, b):
    """Merge two in-flight queues (tuples of (regs, smem, addr)), aligned at the newest entry."""
    if a == b:
        return a
    n = max(len(a), len(b))
    pa, pb = (None,) * (n - len(a)) + a, (None,) * (n - len(b)) + b
    out = []
    for x, y in zip(pa, pb):
        if x is None or y is None:
            out.append(x or y)
        else:
            out.append((x[0] | y[0], x[1] or y[1], min(x[2], y[2])))
    return tuple(out[-QCAP:])


def decode(insn):
    """One instruction, pre-digested for the data-flow pass: (addr, text, waits or None, vm, lgkm,
    smem, registers it will write late, registers it touches now)."""
    addr, mn, ops, _ = insn
    if mn == "s_waitcnt":
        return addr, mn, {c: int(n) for c, n in _WAIT.findall(ops)}, False, False, False, frozenset(), frozenset()
    vm, lgkm, smem, dest = classify(mn, ops)
    touched = _regs(ops, _VREG) | _regs(ops, _SREG)
    if vm and dest and not lgkm:  # a vm load may overwrite an older vm load's target: they return in order
        touched -= dest
    return addr, f"{mn} {ops}".strip(), None, vm, lgkm, smem, frozenset(dest), frozenset(touched)


def _step(state, d, hazards=None, fname=""):
    addr, text, waits, vm, lgkm, smem, dest, touched = d
    vmq, lq = state
    if waits is not None:
        n = waits.get("vmcnt")
        if n is not None and n < len(vmq):
            vmq = vmq[len(vmq) - n:]
        n = waits.get("lgkmcnt")
        if n is not None and n < len(lq) and (n == 0 or not any(e[1] for e in lq)):
            lq = lq[len(lq) - n:]
        return vmq, lq
    if hazards is not None and touched:
        for qi, q in enumerate((vmq, lq)):
            for regs, _, laddr in q:
                hit = (touched | (dest if qi == 1 and vm and not lgkm else frozenset())) & regs
                if hit:
                    hazards.add((fname, addr, text, laddr, tuple(sorted(hit))))
    if vm or lgkm:
        entry = (dest, smem, addr)
        if vm:
            vmq = (vmq + (entry,))[-QCAP:]
        if lgkm:
            lq = (lq + (entry,))[-QCAP:]
    return vmq, lq


def check_function(name, insns):
    """Hazards of one kernel: [(kernel, insn addr, insn, load addr, registers)]."""
    if not insns:
        return []
    dec = [decode(i) for i in insns]
    addrs = [i[0] for i in insns]
    index = {a: k for k, a in enumerate(addrs)}
    leaders = {0}
    for k, (_, mn, _, tgt) in enumerate(insns):
        if tgt is not None and tgt in index:
            leaders.add(index[tgt])
        if tgt is not None or mn in ("s_endpgm", "s_setpc_b64"):
            if k + 1 < len(insns):
                leaders.add(k + 1)
    starts = sorted(leaders)
    blocks = {s: (s, (starts[j + 1] if j + 1 < len(starts) else len(insns))) for j, s in enumerate(starts)}

    def succs(s):
        _, e = blocks[s]
        _, mn, _, tgt = insns[e - 1]
        out = []
        if tgt is not None and tgt in index:
            out.append(index[tgt])
        if mn not in ("s_branch", "s_endpgm", "s_setpc_b64") and e < len(insns):
            out.append(e)
        return out

    empty = ((), ())
    state_in = {0: empty}
    work = [0]
    rounds = 0
    while work:
        rounds += 1
        if rounds > 200000:
            raise RuntimeError(f"asmcheck: no fixpoint in {name}")
        s = work.pop()
        st = state_in[s]
        b, e = blocks[s]
        for k in range(b, e):
            st = _step(st, dec[k])
        for t in succs(s):
            old = state_in.get(t)
            new = st if old is None else (_join(old[0], st[0]), _join(old[1], st[1]))
            if new != old:
                state_in[t] = new
                work.append(t)
    hazards = set()
    for s, st in state_in.items():
        b, e = blocks[s]
        for k in range(b, e):
            st = _step(st, dec[k], hazards, name)
    return sorted(hazards)


def check_library(so_path, arch="gfx950", kernels=None):
    """Every hazard in the code object of so_path (kernels: a name filter, substring match)."""
    funcs = parse(disassemble(so_path, arch))
    out = []
    for name, insns in funcs.items():
        if kernels and not any(k in name for k in kernels):
            continue
        out.extend(check_function(name, insns))
    return out, len(funcs)


def main(argv):
    here = os.path.dirname(os.path.abspath(__file__))
    so = argv[1] if len(argv) > 1 else os.path.join(here, "libgta.so")
    hazards, n = check_library(so)
    for h in hazards[:50]:
        print("HAZARD", h)
    print(f"asmcheck: {n} kernels, {len(hazards)} hazards")
    return 1 if hazards else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
