"""Lists cross-lane reads (rdlane / __shfl / uni) inside `if (ln == 0)` / `if (lane_id() == 0)` regions of a
kernel source: only lane 0 is active there, so a spilled value reloaded inside holds lane 0's bits only.
usage: python scripts/probes/find_lane0_crossreads.py fluidframework_amd/csrc/apply.hip.h"""
import re, sys
src = open(sys.argv[1]).read()
lines = src.split('\n')
pat = re.compile(r'if \((ln|lane_id\(\)) == 0\)')
for i, l in enumerate(lines):
    m = pat.search(l)
    if not m: continue
    rest = l[m.end():]
    if '{' in rest:
        depth = 0; body = []
        for j in range(i, min(i+60, len(lines))):
            seg = lines[j] if j > i else rest
            depth += seg.count('{') - seg.count('}')
            body.append((j+1, lines[j]))
            if depth <= 0 and j > i: break
        for n, b in body:
            if 'rdlane' in b or '__shfl' in b or 'uni(' in b:
                print(f"{i+1}->{n}: {b.strip()}")
    else:
        if 'rdlane' in rest or '__shfl' in rest or 'uni(' in rest:
            print(f"{i+1}: {l.strip()}")
