"""Scan gfx950 assembly for reads of an MFMA result that follow the MFMA too
closely (a dev check for kernels with inline-asm MFMAs, whose results hipcc's
hazard recognizer does not track: CDNA guide, "What hipcc does not do").

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -S --cuda-device-only \
        epfl_megatron_amd/csrc/gemm_nt.hip -o /tmp/gemm_nt.s
    python scripts/asm_hazard_scan.py /tmp/gemm_nt.s [kernel-name-substring]

Per kernel: the fewest instructions / nop states between an MFMA and the
first instruction reading (or rewriting) its destination registers inside
straight-line code, the compiler's AGPR-to-AGPR copies, and the spill count.
A 32x32x16 result needs 12 states before a VALU / accvgpr reader (8 passes),
a 16x16x32 result fewer.  Builtin MFMAs (no inline asm) are covered by the
compiler itself; the count is informative there.
"""
import re,collections,sys
def regs(tok):
    tok=tok.strip()
    m=re.match(r'([va])\[(\d+):(\d+)\]',tok)
    if m: return {(m.group(1),i) for i in range(int(m.group(2)),int(m.group(3))+1)}
    m=re.match(r'([va])(\d+)$',tok)
    if m: return {(m.group(1),int(m.group(2)))}
    return set()
s=open(sys.argv[1]).read()
pat=sys.argv[2] if len(sys.argv)>2 else ''
for fn in re.findall(r'^(_Z[^:\s]*):',s,re.M):
    if pat not in fn: continue
    start=s.index(fn+':'); end=s.find('.Lfunc_end',start)
    body=[l.strip() for l in s[start:end].split('\n') if l.strip() and not l.strip().startswith(';')]
    c=collections.Counter(l.split()[0] for l in body if not l.startswith('.'))
    if not c['v_mfma_f32_32x32x16_bf16'] and not c['v_mfma_f32_16x16x32_bf16']: continue
    worst=(999,None)
    for k,l in enumerate(body):
        if not l.startswith('v_mfma'): continue
        d=regs(l.split(None,1)[1].split(',')[0])
        states=0
        for j in range(k+1,min(k+80,len(body))):
            x=body[j]
            if x.startswith('.LBB'): continue
            if x.startswith('s_nop'): states+=int(x.split()[1])+1; continue
            if x.startswith('v_mfma'):
                if regs(x.split(None,1)[1].split(',')[0])==d: break
                states+=1; continue
            parts=x.split(None,1)
            if len(parts)>1 and (x.startswith('v_') or x.startswith('ds_') or x.startswith('global_') or x.startswith('buffer_')):
                srcs=set()
                for o in parts[1].split(','): srcs|=regs(o)
                if srcs & d:
                    if states<worst[0]: worst=(states,(l[:50],x[:50]))
                    break
            states+=1
    m=re.search(r'\.vgpr_spill_count:\s*(\d+)', s[start:]) 
    print(fn[:80], 'accmov', c['v_accvgpr_mov_b32'], 'min-states', worst[0], worst[1] if worst[0]<12 else '', 'spill', m.group(1) if m else '?')
