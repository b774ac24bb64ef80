"""ISA lint: no instruction reads a VGPR whose vector-memory load is still
outstanding.  The compiler waits for its own loads before any use; an
inline-asm load is "ready" to it when the asm statement ends, so a copy it
inserts before a hand-written counted s_waitcnt reads the register's OLD
value (round 6: nw_align_pka's intermittent wrong penalties,
csrc/nwk_kernels.hip NWK_ASM_PREFETCH).  Follows every branch from each load
until an s_waitcnt vmcnt(N) with N <= the vector-memory ops issued since.
usage: python tools/vmscan.py <file.s> <function symbol>   (prints "<fn> issues K")
"""
import re, sys
lines = open(sys.argv[1]).read().split('\n')
fn = sys.argv[2]
start = next(i for i,l in enumerate(lines) if l.startswith(fn+':'))
end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
body = lines[start:end]
labels = {}
for i,l in enumerate(body):
    m = re.match(r'^(\.?L\w+):', l)
    if m: labels[m.group(1)] = i
def regs_of(op):
    out=[]
    for m in re.finditer(r'\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]', op):
        if m.group(1): out.append(m.group(1)+m.group(2))
        else:
            for r in range(int(m.group(4)), int(m.group(5))+1): out.append(m.group(3)+str(r))
    return out
VM = ('global_load','global_store','global_atomic','buffer_load','buffer_store','buffer_atomic','scratch_load','scratch_store','flat_')
LD = ('global_load','buffer_load','scratch_load')
issues=[]
for i,l in enumerate(body):
    s=l.strip()
    if not s.startswith(LD) or 'lds' in s.split()[0]: continue
    dst=set(regs_of(s.split(None,1)[1].split(',')[0]))
    stack=[(i+1,0)]; seen=set()
    found=None
    steps=0
    while stack and not found and steps < 200000:
        j,cnt = stack.pop()
        while j < len(body):
            steps+=1
            if (j,cnt) in seen: break
            seen.add((j,cnt))
            t=body[j].strip()
            if not t or t.startswith(';') or t.startswith('.') or re.match(r'^\.?L\w+:', t):
                j+=1; continue
            op=t.split(None,1)
            if op[0]=='s_waitcnt':
                m=re.search(r'vmcnt\((\d+)\)', t)
                if m and int(m.group(1)) <= cnt: break
                j+=1; continue
            if op[0] in ('s_endpgm','s_setpc_b64'): break
            if op[0]=='s_branch':
                tgt=op[1].strip(); 
                if tgt in labels: j=labels[tgt]; continue
                break
            if op[0].startswith('s_cbranch'):
                tgt=op[1].strip()
                if tgt in labels: stack.append((labels[tgt],cnt))
                j+=1; continue
            if op[0].startswith('s_swappc') or op[0].startswith('s_call'):
                break
            srcs=[]
            if op[0].startswith(VM):
                srcs = op[1].split(',')[1:] if op[0].startswith(LD) else op[1].split(',')
                cnt=min(cnt+1, 64)
            elif len(op)>1:
                srcs = op[1].split(',')[1:]
            sr=set()
            for x in srcs: sr.update(regs_of(x))
            if sr & dst:
                found=(j,t,cnt); break
            # dst overwritten by another instruction (not reading): kill tracking of those regs
            if len(op)>1 and not op[0].startswith(VM):
                d=set(regs_of(op[1].split(',')[0]))
                if d & dst and d >= dst: break
            j+=1
    if found:
        issues.append((start+i+1, s, start+found[0]+1, found[1], found[2]))
for x in issues[:20]: print(x)
print(fn, 'issues', len(issues))
