#!/usr/bin/env python3
"""CPU simulation of k_map's LDS key table on one workgroup's share of the C2 corpus (4 MiB, ~709 K
tokens): hit rate of the best static table (the most frequent 8,410 short and 1,024 medium keys)
against 2-choice slots with second-sight admission (the kernel's policy) and variants (more
choices, admission on third sight).  Usage: tools/hit_sim.py [bytes]   (r06; CPU only, seconds)"""
import os
import sys, re, collections, random
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'mit-6.824-2015_amd'))
from wcg.corpus import Generator, CONFIGS
cfg=CONFIGS['c2_ascii_zipf_1gib']
g=Generator(cfg['mode'],cfg['vocab'],cfg['zipf_s'],cfg['seed'])
nb=int(sys.argv[1]) if len(sys.argv)>1 else 4<<20
data=g.bytes(nb, first_block=37)
toks=re.findall(rb'[A-Za-z]+', data)
print('tokens',len(toks))
short=[t for t in toks if len(t)<=7]; med=[t for t in toks if 8<=len(t)<=15]
print('short',len(short),'med',len(med),'long',len(toks)-len(short)-len(med))
NS,NM=8410,1024
def opt(lst,n):
    c=collections.Counter(lst); return sum(v for _,v in c.most_common(n))
print('optimal static hits', (opt(short,NS)+opt(med,NM))/len(toks))
R=random.Random(1)
hs={}
def H(t):
    h=hs.get(t)
    if h is None: h=hs[t]=R.getrandbits(64)
    return h
def sim(lst,n,choices=2,admit_bits=16384,admit_need=1):
    tab=[None]*n; seen=collections.Counter() if admit_bits else None
    hits=0
    for t in lst:
        h=H(t)
        cand=[(h>>(i*20))%n for i in range(choices)]
        if any(tab[c]==t for c in cand): hits+=1; continue
        free=[c for c in cand if tab[c] is None]
        if not free: continue
        if seen is not None:
            b=(h>>50)%admit_bits
            seen[b]+=1
            if seen[b]<=admit_need: continue
        tab[free[0]]=t; hits+=1
    return hits
for ch,ab,an in [(2,16384,1),(2,0,0),(4,16384,1),(2,16384,2),(4,16384,2),(8,16384,1)]:
    hsum=sim(short,NS,ch,ab,an)+sim(med,NM,ch,ab,an)
    print('choices',ch,'admit bits',ab,'need',an,'hit',round(hsum/len(toks),4))
