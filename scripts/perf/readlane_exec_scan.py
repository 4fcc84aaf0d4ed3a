#!/usr/bin/env python3
"""Scan a device assembly function (hipcc --cuda-device-only -S, one function
extracted) for v_readlane_b32 with an SGPR lane index whose source VGPR was
written after the innermost exec-mask change (s_and_saveexec / s_mov exec):
an exec-masked copy leaves the inactive lanes stale, and readlane of such a
lane reads garbage. Usage: readlane_exec_scan.py FUNC.s"""
import re,sys
lines=open(sys.argv[1]).read().splitlines()
n=0; ex=[]
for j,l in enumerate(lines):
    r=re.match(r"\s+v_readlane_b32 s\d+, (v\d+), (s\d+)$",l)
    if not r: continue
    v=r.group(1)
    # walk back to the innermost exec change
    k=j-1
    while k>0 and not re.match(r"\s+(s_and_saveexec_b64|s_mov_b64 exec|s_or_b64 exec|s_andn2_b64 exec|s_and_b64 exec|s_xor_b64 exec)",lines[k]):
        k-=1
    if not lines[k].strip().startswith("s_and_saveexec") and "s_mov_b64 exec" not in lines[k]: continue
    for m in range(k+1,j):
        d=re.match(r"\s+(v_\w+|ds_read\w*)\s+(v\[(\d+):(\d+)\]|v(\d+))",lines[m])
        if d and not lines[m].strip().startswith(("v_readlane","v_cmp","v_writelane")):
            regs = range(int(d.group(3)),int(d.group(4))+1) if d.group(3) else [int(d.group(5))]
            if int(v[1:]) in regs:
                n+=1
                if n<=4: print(f"line {j+1}: {l.strip()} <- line {m+1}: {lines[m].strip()} (exec set at line {k+1}: {lines[k].strip()})")
                ex.append(j); break
print("readlanes of a VGPR written under the current partial exec:",n)
