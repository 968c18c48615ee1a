"""Compile pcabi_engine.hip for gfx950 with -save-temps and report, per k_align instantiation,
VGPR/SGPR/occupancy and the VALU instruction count of the hottest loop (column loop)."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, 'custom_porechop_abi_amd', 'csrc', 'pcabi_engine.hip')
want = sys.argv[1:] or ['24', '32', '48']
tmp = tempfile.mkdtemp()
subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '--save-temps',
                '-c', SRC, '-o', os.path.join(tmp, 'x.o')], cwd=tmp, check=True,
               stderr=subprocess.DEVNULL)
asm = open(os.path.join(tmp, 'pcabi_engine-hip-amdgcn-amd-amdhsa-gfx950.s')).read()
for rpl in want:
    for aff in ('1', '0'):
        name = '_ZN12_GLOBAL__N_17k_alignILi%sELb%sELi0EEEvNS_7KParamsE' % (rpl, aff)
        i = asm.find(name + ':')
        if i < 0:
            continue
        body = asm[i:asm.find('.Lfunc_end', i)]
        meta = asm[asm.find('.name:           ' + name):]
        vg = re.search(r'\.vgpr_count:\s+(\d+)', meta[:3000] if meta else '')
        sg = re.search(r'\.sgpr_count:\s+(\d+)', meta[:3000] if meta else '')
        # loops: find backward branches; take the largest block between a label and its branch back
        lines = body.split('\n')
        labels = {l.split(':')[0]: k for k, l in enumerate(lines) if re.match(r'^\.LBB\d+_\d+:', l)}
        best = (0, None)
        for k, l in enumerate(lines):
            m = re.search(r's_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)', l)
            if m:
                tgt = m.group(1) or m.group(2)
                if tgt in labels and labels[tgt] < k:
                    seg = lines[labels[tgt]:k + 1]
                    nv = sum(1 for x in seg if re.match(r'\s+v_', x))
                    if nv > best[0]:
                        best = (nv, seg)
        mix = {}
        for x in best[1] or []:
            mm = re.match(r'\s+(v_\w+)', x)
            if mm:
                mix[mm.group(1)] = mix.get(mm.group(1), 0) + 1
        top = sorted(mix.items(), key=lambda t: -t[1])[:12]
        print('RPL=%s affine=%s vgpr=%s sgpr=%s loopVALU=%d (%.2f/row) %s' % (
            rpl, aff, vg.group(1) if vg else '?', sg.group(1) if sg else '?', best[0], best[0] / float(rpl), top))
