"""Instruction mix and register counts of kernels in a hipcc -S device assembly file.
usage: python tools/isa_mix.py file.s name_substring"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
for m in re.finditer(r'^(_Z\S*' + re.escape(sys.argv[2]) + r'\S*):', s, re.M):
    name = m.group(1)
    a = m.end()
    b = s.index('.Lfunc_end', a)
    body = s[a:b]
    ins = [l.strip().split()[0] for l in body.split('\n') if l.startswith('\t') and not l.strip().startswith(('.', ';'))]
    c = Counter(ins)
    vg = re.search(r'NumVgprs:\s+(\d+)', s[b:b + 5000]); sg = re.search(r'NumSgprs:\s+(\d+)', s[b:b + 5000])
    print(name[:60], 'vgpr', vg.group(1) if vg else '?', 'sgpr', sg.group(1) if sg else '?', 'instrs', len(ins),
          'readlane', c['v_readlane_b32'], 'writelane', c['v_writelane_b32'], 'nop', c['s_nop'],
          'cndmask', c['v_cndmask_b32_e64'] + c['v_cndmask_b32_e32'], 'med3', c['v_med3_u32'],
          'saveexec', c['s_and_saveexec_b64'], 'bperm', c['ds_bpermute_b32'], 'sgpr-spill', body.count('SGPR spill'))
