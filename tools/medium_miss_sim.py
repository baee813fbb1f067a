#!/usr/bin/env python3
"""CPU check of the medium-key miss buckets (r06): lds_hash and k_map's slot choices restated in
Python for the C2 corpus's most frequent medium keys, then one workgroup's medium stream through a
1,024-slot 2-choice table with second-sight admission (the real hash and slot functions); prints,
per medium miss bucket, the share of its units taken by its most-missed key.  Usage:
tools/medium_miss_sim.py   (CPU only, seconds)"""
import os
import sys, re, collections
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'mit-6.824-2015_amd'))
from wcg.corpus import Generator, CONFIGS
M=0xFFFFFFFF
def rotl(x,r): return ((x<<r)|(x>>(32-r)))&M
def lds_hash32(a,b,c,d):
    x=a^rotl(b,9)^rotl(c,17)^rotl(d,25)
    x^=x>>15; x=(x*0x2C1B3C6D)&M; x^=x>>12; return x
def key(t):
    L=len(t)
    if L<=7:
        k0=int.from_bytes(t,'little')|(L<<56); k1=0
    else:
        k0=int.from_bytes(t[:8],'little'); k1=int.from_bytes(t[8:],'little')|(L<<56)
    return k0,k1
def h(t):
    k0,k1=key(t); return lds_hash32(k0&M,k0>>32,k1&M,k1>>32)
def slots(hh,n):
    return (((hh>>8)*(n<<8))>>32, ((hh&0xFFFFFF)*(n<<8))>>32)
cfg=CONFIGS['c2_ascii_zipf_1gib']
g=Generator(cfg['mode'],cfg['vocab'],cfg['zipf_s'],cfg['seed'])
data=g.bytes(4<<20, first_block=37)
toks=re.findall(rb'[A-Za-z]+', data)
med=[t for t in toks if 8<=len(t)<=15]
c=collections.Counter(med)
top=c.most_common(40)
slotmap=collections.defaultdict(list)
for t,v in c.most_common(3000):
    for s in slots(h(t),1024): slotmap[s].append((t,v))
for t,v in top[:12]:
    hh=h(t); s=slots(hh,1024)
    print(t, v, 'bucket', (hh&31)+64, 'slots', s, [ (x[0],x[1]) for ss in s for x in slotmap[ss] if x[0]!=t][:4])
print('---- k_map medium table simulation (real slots, admission)')
NM=1024
tab=[None]*NM; seen=set(); miss=collections.Counter()
for t in med:
    hh=h(t); s1,s2=slots(hh,NM)
    if tab[s1]==t or tab[s2]==t: continue
    if tab[s1] is None or tab[s2] is None:
        b=((hh*0x9E3779B1)&M)>>18
        if b in seen:
            if tab[s1] is None: tab[s1]=t
            else: tab[s2]=t
            continue
        seen.add(b)
    miss[t]+=1
tot=sum(miss.values()); print('misses',tot,'rate',tot/len(med))
byb=collections.defaultdict(collections.Counter)
for t,v in miss.items(): byb[(h(t)&31)+64][t]+=v
rows=[]
for b,cn in byb.items():
    s=sum(cn.values()); k,v=cn.most_common(1)[0]
    rows.append((v/s, b, s, k, v))
rows.sort(reverse=True)
for r in rows[:6]: print('bucket',r[1],'units',r[2],'top key',r[3],r[4],'share',round(r[0],3))
print('median share', sorted(r[0] for r in rows)[len(rows)//2])
