#!/usr/bin/env python3
"""Dev tool: how far a Huffman walk started at an arbitrary bit of a config-3 literal runs before it
falls into step with the true walk (the resync distance that bounds speculative segment decoding).
Prints the fraction of 13k random starts synchronised within 16..128 bits."""
import numpy as np, sys
sys.path.insert(0,'/root/repo')
from loona_amd import synth
from loona_amd.huffman import huffman_encode
L = synth.code_lengths()
# build code table
import itertools
codes={}
order=sorted(range(257), key=lambda s:( [*L,30][s] if s<256 else 30, s))
lens=list(L)+[30]
c=0; prev=lens[order[0]]
code=[0]*257
for i,s in enumerate(order):
    l=lens[s]
    if i: c=(c+1)<<(l-prev)
    prev=l; code[s]=c
dec={ (lens[s],code[s]): s for s in range(257)}
def boundaries(bits, start, end):
    # walk from start, return list of code start positions (stop at end or invalid/EOS)
    p=start; out=[]
    n=len(bits)
    while p < end:
        v=0
        for l in range(1,31):
            if p+l>n: return out, None
            v=(v<<1)|bits[p+l-1]
            if (l,v) in dec:
                s=dec[(l,v)]
                out.append(p)
                if s==256: return out, 'eos'
                p+=l; break
        else:
            return out, 'bad'
    return out, None
rng=np.random.default_rng(1)
w=synth.config3(n=3000)
res=[]
for i in range(w.n):
    a,b=int(w.enc_off[i]),int(w.enc_off[i+1])
    if b-a<256: continue
    data=w.enc_blob[a:b]
    bits=np.unpackbits(data).tolist()
    true,_=boundaries(bits,0,len(bits))
    ts=set(true)
    for _ in range(20):
        s=int(rng.integers(1,len(bits)-400))
        bs,_=boundaries(bits,s,s+300)
        # sync distance: first boundary in bs that is a true boundary
        d=None
        for p in bs:
            if p in ts: d=p-s; break
        res.append(d if d is not None else 9999)
r=np.array(res)
for L_ in [16,24,32,48,64,96,128]:
    print(L_, (r<=L_).mean())
print('n',len(r), 'max', r[r<9999].max(), 'fail', (r==9999).sum())
