"""Static audit of the hand-written LDS-DMA / vmcnt sites in the gfx950 ISA.

usage: python tools/asm_audit.py BUILD_DIR   (BUILD_DIR holds the *-hip-amdgcn-amd-amdhsa-gfx950.s
files of `hipcc -save-temps`; tools/asm_audit.sh builds them)

For every kernel that contains an inline-asm `global_load_lds_dwordx4` / `_dword` it reports:
  * .vgpr_spill_count, .sgpr_spill_count, .private_segment_fixed_size (scratch) from the
    kernel descriptor metadata;
  * hazard H1 (cdna_hip_programming.md §5.7 item 2): an SGPR used as the DMA's saddr that a
    VALU instruction (v_readfirstlane_b32 / v_readlane_b32 / v_cmp* writing an SGPR) wrote
    fewer than 5 wait states before the DMA (VALU SGPR write -> VMEM SGPR read needs 5);
    the asm string itself provides the states of its own instructions before the DMA;
  * hazard H2: `s_mov_b32 m0, ...` followed by the DMA without a wait state in between;
  * every inline-asm `s_waitcnt vmcnt(N)`: the VMEM instructions issued on the straight-line
    path since the previous wait / barrier of the same kind, youngest first, so that the
    claim "the N youngest are the next chunk's DMAs" can be checked site by site
    (a DMA issued conditionally under `s_cbranch_execz` would not count).
"""

from __future__ import annotations

import re
import sys
from pathlib import Path

VMEM = re.compile(r"^\s*(global_load|global_store|buffer_load|buffer_store|global_atomic|buffer_atomic|flat_)")
SGPR_WRITE_VALU = re.compile(r"^\s*(v_readfirstlane_b32|v_readlane_b32|v_cmp\w*|v_cmpx\w*|v_div_scale\w*|"
                             r"v_add_co_u32|v_sub_co_u32|v_addc_co_u32|v_subb_co_u32)\s+(s\[?\d+(:\d+)?\]?|vcc)")
SREG = re.compile(r"s\[(\d+):(\d+)\]|s(\d+)")


def sregs(tok: str) -> set[int]:
    out = set()
    for m in SREG.finditer(tok):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def kernels(text: str):
    """(name, body lines, metadata dict) per kernel in an .s file"""
    meta = {}
    for m in re.finditer(r"\.name:\s+(\S+)\n(?:.*\n)*?", text):
        pass
    # metadata block: "- .agpr_count ... .name: X ... .private_segment_fixed_size: N ... .vgpr_spill_count: N"
    for blk in re.split(r"\n  - \.", text.split("amdhsa.kernels:")[-1])[1:]:
        nm = re.search(r"\.name:\s+(\S+)", blk)
        if not nm:
            continue
        d = {}
        for key in ("private_segment_fixed_size", "vgpr_spill_count", "sgpr_spill_count", "group_segment_fixed_size",
                    "vgpr_count", "agpr_count"):
            mm = re.search(r"\." + key + r":\s+(\d+)", blk)
            if mm:
                d[key] = int(mm.group(1))
        meta[nm.group(1)] = d
    for m in re.finditer(r"^(\S+):\s*; @\S+\n(.*?)^\s*s_endpgm", text, re.S | re.M):
        name = m.group(1)
        if name.startswith(".") or name not in meta:
            continue
        yield name, m.group(2).split("\n"), meta[name]


def instr(line: str) -> str | None:
    s = line.strip()
    if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
        return None
    return s.split(";")[0].strip() or None


def audit(path: Path):
    text = path.read_text()
    rows = []
    for name, lines, meta in kernels(text):
        if "global_load_lds_dword" not in "\n".join(lines):
            continue
        seq = []  # (instr, in_asm)
        in_asm = False
        for ln in lines:
            s = ln.strip()
            if s.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if s.startswith(";;#ASMEND"):
                in_asm = False
                continue
            if s.endswith(":") and not s.startswith(";"):
                seq.append((s, False, True))  # label
                continue
            i = instr(ln)
            if i:
                seq.append((i, in_asm, False))
        h1, h2, waits = [], [], []
        ndma = 0
        for k, (ins, asm, lab) in enumerate(seq):
            if lab:
                continue
            if asm and ins.startswith("global_load_lds_dword"):
                ndma += 1
                ops = [t.strip() for t in ins.split(None, 1)[1].split(",")]
                sbase = sregs(ops[1]) if len(ops) > 1 and ops[1] != "off" else set()
                # H2: m0 write immediately before
                prev = [x for x in seq[max(0, k - 3):k] if not x[2]]
                if prev and prev[-1][0].startswith("s_mov_b32 m0"):
                    h2.append(ins)
                # H1: walk back counting wait states until a VALU write of a base SGPR
                states = 0
                for j in range(k - 1, max(-1, k - 40), -1):
                    p, _, plab = seq[j]
                    if plab:
                        break  # do not cross block boundaries (reported separately if needed)
                    mnop = re.match(r"s_nop\s+(\d+)", p)
                    if mnop:
                        states += int(mnop.group(1)) + 1
                        continue
                    w = SGPR_WRITE_VALU.match(p)
                    if w and (sregs(w.group(2)) & sbase):
                        if states < 5:
                            h1.append((ins, p, states))
                        break
                    states += 1
                    if states >= 5:
                        break
            if asm and re.match(r"s_waitcnt\s+vmcnt\((\d+)\)", ins):
                n = int(re.match(r"s_waitcnt\s+vmcnt\((\d+)\)", ins).group(1))
                younger = []
                for j in range(k - 1, -1, -1):
                    p, pasm, plab = seq[j]
                    if plab:
                        younger.append("<label>")
                        continue
                    if p.startswith("s_cbranch") or p.startswith("s_branch"):
                        younger.append("<" + p.split()[0] + ">")
                        continue
                    if (pasm and p.startswith("s_waitcnt") and "vmcnt" in p) or p.startswith("s_barrier"):
                        if len([y for y in younger if y not in ("<label>",)]) >= n or p.startswith("s_waitcnt"):
                            break
                    if VMEM.match(p):
                        younger.append(("DMA" if (pasm and "lds" in p) else p.split()[0]))
                    if len([y for y in younger if not y.startswith("<")]) > n + 8:
                        break
                waits.append((n, younger[:n + 8]))
        rows.append((name, meta, ndma, h1, h2, waits))
    return rows


def main():
    d = Path(sys.argv[1] if len(sys.argv) > 1 else "/tmp/audit")
    bad = 0
    for s in sorted(d.glob("*-hip-amdgcn-amd-amdhsa-gfx950.s")):
        for name, meta, ndma, h1, h2, waits in audit(s):
            short = name if len(name) < 90 else name[:87] + "..."
            print(f"{s.name.split('-hip')[0]:10s} {short}")
            print(f"    DMAs {ndma}, scratch {meta.get('private_segment_fixed_size')} B, vgpr spill "
                  f"{meta.get('vgpr_spill_count')}, sgpr spill {meta.get('sgpr_spill_count')}, static LDS "
                  f"{meta.get('group_segment_fixed_size')} B, VGPR {meta.get('vgpr_count')} AGPR {meta.get('agpr_count')}")
            for ins, p, st in h1:
                bad += 1
                print(f"    H1 HAZARD: {p!r} -> {ins!r} after {st} wait states (< 5)")
            for ins in h2:
                bad += 1
                print(f"    H2 HAZARD: m0 write directly before {ins!r}")
            for n, y in waits:
                # the walk back to the n-th youngest VMEM op: straight-line when no branch lies on it
                ops, walked = 0, []
                for t in y:
                    walked.append(t)
                    if not t.startswith("<"):
                        ops += 1
                        if ops >= n:
                            break
                branches = [t for t in walked if t.startswith("<s_")]
                nondma = [t for t in walked if not t.startswith("<") and t != "DMA"]
                if ops < n:
                    tag = "CHECK(short)"
                elif branches:
                    tag = "CHECK(branch)"
                elif nondma:
                    tag = "ok(+loads)"
                else:
                    tag = "ok "
                print(f"    vmcnt({n}) {tag} youngest-first: {' '.join(t if isinstance(t, str) else t for t in y)}")
    print(f"hazards: {bad}")


if __name__ == "__main__":
    main()
