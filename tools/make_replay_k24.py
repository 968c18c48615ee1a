"""Generate the replay microbenchmark of the dominant kernel's inner column.

Compiles the kernel translation unit that holds k_align<24, true, TAGGED> (the headline's dominant
launch) to gfx950 assembly, extracts that kernel's inner column loop -- the blocks of the loop with
the most v_max3_i32, i.e. LanePacked::column over 24 adapter rows, the window reader's look-ahead
load every 4 columns and the row-L scout -- VERBATIM, and writes:

  profiles/r05/k_align24_inner_column.s   the loop as the compiler emitted it (labels as emitted)
  tools/replay_k24_body.inc               the same text as C string literals for tools/replay_k24.hip,
                                          labels renamed, one copy per variant:
                                            exact   -- the loop as emitted
                                            nolds   -- the ds_reads and their lgkmcnt waits removed
                                                       (the destinations keep stale values): the
                                                       VALU + SALU issue of the same mix alone

Run: python tools/make_replay_k24.py   (hipcc, ~20 s), then build tools/replay_k24.hip.
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = '_ZN9pcabi_eng7k_alignILi24ELb1ELi6EEEvNS_7KParamsE'


def device_asm():
    out = os.path.join(ROOT, 'build', 'replay', 'pcabi_k_packed_small.s')
    os.makedirs(os.path.dirname(out), exist_ok=True)
    src = os.path.join(ROOT, 'custom_porechop_abi_amd', 'csrc', 'pcabi_k_packed_small.hip')
    subprocess.check_call(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '--cuda-device-only', '-O3', '-std=c++17',
                           '-S', '-o', out, src])
    return open(out).read().splitlines()


def kernel_lines(lines):
    start = next(i for i, l in enumerate(lines) if l.startswith(KERNEL + ':'))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith('.Lfunc_end') or
               (lines[i].startswith('_Z') and lines[i].rstrip().endswith(':') and i > start + 1))
    return lines[start:end]


def blocks(body):
    """(label, header-of-loop or None, is_header, lines) per basic block."""
    out = []
    cur = None
    for l in body:
        m = re.match(r'^(\.LBB\d+_\d+|; %bb\.\d+):?\s*(.*)$', l)
        if m:
            lab = m.group(1).replace('; %bb.', '.LBB_bb')
            note = m.group(2)
            hdr = re.search(r'Header=BB(\d+_\d+)', note)
            is_h = 'Inner Loop Header' in note
            cur = [lab, hdr.group(1) if hdr else None, is_h, [l]]
            out.append(cur)
        elif cur is not None:
            cur[3].append(l)
    return out


def inner_loop(body):
    """The cross-mode column loop: 24 v_max3_i32 (one per adapter row) and the window reader's
    look-ahead at a runtime stride (the tile layout's 256 dwords, v_mad_u64_u32). The compiler also
    emits a copy of the loop for pairs mode (stride 1, the window's own bytes); that one is not the
    headline's."""
    bl = blocks(body)
    found = []
    for k, b in enumerate(bl):
        if not b[2]:
            continue
        hid = b[0].replace('.LBB', '')
        members = [x for x in bl if x is b or x[1] == hid]
        n3 = sum(l.count('v_max3_i32') for x in members for l in x[3])
        strided = any('v_mad_u64_u32' in l for x in members for l in x[3])
        if n3 == 24 and strided:
            found.append((members, hid))
    if len(found) != 1:
        raise SystemExit('expected one strided 24-row column loop, found %d' % len(found))
    return found[0]


def main():
    lines = device_asm()
    body = kernel_lines(lines)
    members, hid = inner_loop(body)
    text = [l for b in members for l in b[3]]
    # REPLAY_S: where the extracted loop goes (r05: profiles/r05/k_align24_inner_column.s, the loop the
    # replay harness's register setup is written for)
    out_s = os.environ.get('REPLAY_S', os.path.join(ROOT, 'profiles', 'r05', 'k_align24_inner_column.s'))
    os.makedirs(os.path.dirname(out_s), exist_ok=True)
    with open(out_s, 'w') as f:
        f.write('; %s: inner column loop (header .LBB%s), gfx950, hipcc -O3, extracted by '
                'tools/make_replay_k24.py\n' % (KERNEL, hid))
        f.write('\n'.join(text) + '\n')
    labels = sorted({b[0] for b in members})
    exits = sorted({m for l in text for m in re.findall(r'(\.LBB\d+_\d+)', l)} - set(labels))
    if len(exits) != 1:
        raise SystemExit('expected one exit label, found %s' % exits)
    counts = {}
    for l in text:
        m = re.match(r'^\s+([a-z][a-z0-9_]*)', l)
        if m:
            counts[m.group(1)] = counts.get(m.group(1), 0) + 1
    vregs = sorted({int(x) for l in text for x in re.findall(r'\bv(\d+)\b', l)} |
                   {int(a) + i for l in text for a, b in re.findall(r'\bv\[(\d+):(\d+)\]', l)
                    for i in range(int(b) - int(a) + 1)})
    sregs = sorted({int(x) for l in text for x in re.findall(r'\bs(\d+)\b', l)} |
                   {int(a) + i for l in text for a, b in re.findall(r'\bs\[(\d+):(\d+)\]', l)
                    for i in range(int(b) - int(a) + 1)})

    nv = max(vregs) + 1                        # the interleaved copy's registers start here
    lits = {}                                  # VOP2 literal -> SGPR (variant sgprlit)

    def rename(s, k):
        """Copy B of a vector instruction: every VGPR vN -> v(N + k)."""
        s = re.sub(r'\bv\[(\d+):(\d+)\]', lambda m: 'v[%d:%d]' % (int(m.group(1)) + k, int(m.group(2)) + k), s)
        return re.sub(r'\bv(\d+)\b', lambda m: 'v%d' % (int(m.group(1)) + k), s)

    def split3(s, op):
        """v_max3_i32 d, a, b, c -> two VOP2 `op`s (src1 a VGPR; d may alias one source)."""
        m = re.match(r'^\s*v_max3_i32\s+(\S+),\s*(\S+),\s*(\S+),\s*(\S+)$', s)
        d, a, b, c = m.groups()
        srcs = [a, b, c]
        z = next((x for x in srcs if x.startswith('s') and x != d), None) or next(x for x in reversed(srcs) if x != d)
        rest = list(srcs)
        rest.remove(z)
        x, y = rest if rest[1].startswith('v') else (rest[1], rest[0])
        return ['%s %s, %s, %s' % (op, d, x, y), '%s %s, %s, %s' % (op, d, z, d)]

    def variant(tag, mode):
        """mode: exact | nolds (ds_reads and their waits dropped) | nowait (ds_reads kept, waits
        dropped) | sgprlit (VOP2 literals from SGPRs: half the bytes) | max3split (each v_max3_i32
        as two v_max_i32) | maxadd (every max as full-rate v_add_u32s: same chains, no max) |
        inter2 (a second copy of every vector instruction on registers v+NV, interleaved one by
        one: two independent columns per lane, the loop control shared)"""
        out = []
        for l in text:
            s = l.split(';')[0].rstrip()
            if not s.strip():
                continue
            m = re.match(r'^(\.LBB\d+_\d+|; %bb\.\d+)', l)
            if m:
                if m.group(1).startswith('; %bb'):
                    continue                   # fall-through block: no label needed
                out.append(m.group(1).replace('.LBB', '.Lrp_%s_' % tag) + ':')
                continue
            s = s.replace(exits[0], '.Lrp_%s_exit' % tag)
            s = re.sub(r'\.LBB(\d+_\d+)', lambda mm: '.Lrp_%s_%s' % (tag, mm.group(1)), s)
            s = s.strip()
            if mode == 'nolds' and ('ds_read' in s or 'lgkmcnt' in s):
                continue                       # no LDS read, no wait: the destinations keep old values
            if mode == 'nolds_mov' and 'lgkmcnt' in s:
                continue
            if mode == 'nolds_mov' and s.startswith('ds_read'):
                # a fresh value from a register no recent VALU wrote (v70 / v71: the quad read's
                # destinations, never written in this variant): exact's dependency pattern, no LDS
                m2 = re.match(r'^ds_read_b(32|64)\s+(v\d+|v\[\d+:\d+\]),', s)
                dst = m2.group(2)
                if m2.group(1) == '64':
                    continue
                out.append('v_mov_b32_e32 %s, v71' % dst)
                continue
            if mode == 'nowait' and 'lgkmcnt' in s:
                continue
            if mode == 'sgprlit' and s.startswith('v_') and '_e32' in s:
                mm = re.search(r',\s*(0x[0-9a-f]+),', s)
                if mm:
                    reg = lits.setdefault(mm.group(1), 's%d' % (61 + len(lits)))
                    s = s.replace(mm.group(1), reg, 1)
            if mode in ('max3split', 'maxadd') and s.startswith('v_max3_i32'):
                out += split3(s, 'v_max_i32_e32' if mode == 'max3split' else 'v_add_u32_e32')
                continue
            if mode == 'vgconst':               # the cell's SGPR constants read from VGPRs v72 / v73
                s = re.sub(r'^(v_\w+_e32 v\d+), s16,', r'\1, v72,', s)
                s = re.sub(r'^(v_\w+_e32 v\d+), s28,', r'\1, v73,', s)
            if mode == 'maxadd' and s.startswith('v_max_i32'):
                s = s.replace('v_max_i32', 'v_add_u32')
            out.append(s)
            if mode == 'inter2' and re.match(r'^(v_|ds_|global_)', s):
                out.append(rename(s, nv))
        header = '.Lrp_%s_%s' % (tag, hid)
        return header, out

    def half_rate(s):
        """Issue classes measured by tools/replay_k24.hip's rate probes: VOP3 forms and the 32-bit
        maxes take two full-rate issue slots (4 cycles per wave64 instruction)."""
        op = s.split()[0]
        return op.startswith('v_max') or (op.startswith('v_') and not op.endswith(('_e32', '_e64')) and
                                           not op.startswith(('v_mov_b32', 'v_cndmask', 'v_cmp')))

    inc = ['// generated by tools/make_replay_k24.py from %s (do not edit)' % KERNEL,
           '// instruction counts per loop pass: ' + ', '.join('%s %d' % kv for kv in sorted(counts.items())),
           '#define RP_VREGS_MAX %d' % max(vregs),
           '#define RP_NV %d' % nv,
           '#define RP_SREGS_MAX %d' % max(sregs),
           '#define RP_CLOBBER_V %s' % ', '.join('"v%d"' % v for v in range(0, nv)),
           '#define RP_CLOBBER_V2 %s' % ', '.join('"v%d"' % v for v in range(nv, 2 * nv)),
           '#define RP_CLOBBER_S %s' % ', '.join('"s%d"' % s for s in sregs),
           '#define RP_SREGS "%s"' % ' '.join('s%d' % s for s in sregs)]
    load_labels = {b[0].replace('.LBB', '') for b in members if b[0].startswith('.LBB_bb')}
    # the *4 copies run at the other 4-byte code phase (same instructions, own labels)
    for tag, mode in (('exact', 'exact'), ('nolds', 'nolds'), ('nowait', 'nowait'), ('sgprlit', 'sgprlit'),
                      ('max3split', 'max3split'), ('maxadd', 'maxadd'), ('inter2', 'inter2'), ('exact4', 'exact'),
                      ('nolds4', 'nolds'), ('vgconst', 'vgconst'), ('nolds_mov', 'nolds_mov')):
        header, out = variant(tag, mode)
        inc.append('#define RP_HEADER_%s "%s"' % (tag.upper(), header))
        inc.append('#define RP_EXIT_%s ".Lrp_%s_exit:\\n"' % (tag.upper(), tag))
        inc.append('#define RP_LOOP_%s \\' % tag.upper())
        for s in out:
            inc.append('    "%s\\n" \\' % s.replace('\t', ' ').strip())
        inc.append('    ""')
        # per pass: VALU of the main blocks, VALU of the look-ahead block (every 4th pass), and
        # how many of the main blocks' VALU are half rate
        main, load, half = 0, 0, 0
        in_load = False
        for s in out:
            if s.endswith(':'):
                continue
            if s.startswith('s_lshr_b32'):     # the look-ahead block's first instruction
                in_load = True
            if s.startswith('s_branch') and in_load:
                in_load = False
                continue
            if s.startswith('v_'):
                if in_load:
                    load += 1
                else:
                    main += 1
                    half += half_rate(s)
        inc.append('#define RP_VALU_MAIN_%s %d' % (tag.upper(), main))
        inc.append('#define RP_VALU_LOAD_%s %d' % (tag.upper(), load))
        inc.append('#define RP_VALU_HALF_%s %d' % (tag.upper(), half))
    inc.append('#define RP_SGPRLIT_SETUP "%s"' % ''.join('s_mov_b32 %s, %s\\n' % (r, v) for v, r in lits.items()))
    inc.append('#define RP_CLOBBER_LIT %s' % ', '.join('"%s"' % r for r in lits.values()))
    valu = sum(v for k, v in counts.items() if k.startswith('v_'))
    if os.environ.get('REPLAY_NO_INC') == '1':    # extraction only (ISA of the current source)
        return 0
    # tools/replay_k24.hip's register setup (RP_SETUP) is written for the r05 loop (the source at
    # faa8f29): LDS row stride in s57, table base in v16, constants in s16 / s28. Refuse another.
    if not any('v_mad_u32_u24 v0, v0, s57, v16' in l for l in text):
        raise SystemExit('this loop is not the r05 one the replay setup is written for: build it from the r05 '
                         'source (git show faa8f29:custom_porechop_abi_amd/csrc/pcabi_dp.h) or use REPLAY_NO_INC=1')
    with open(os.path.join(ROOT, 'tools', 'replay_k24_body.inc'), 'w') as f:
        f.write('\n'.join(inc) + '\n')
    print('loop header .LBB%s: %d lines, %d VALU per pass, exits to %s; vregs up to v%d, sregs %s' % (
        hid, len(text), valu, exits[0], max(vregs), sregs))
    print(sorted(counts.items()))


if __name__ == '__main__':
    sys.exit(main())
