"""Development study (CPU): speculative starts for __sort_heap's pipelined pops (tools/mb/heap_pop.hip
pops_v41). One pop in flight per lane of a wave, a start every two steps; v40 (the library's engine)
starts a pop only when no older hole is its last element q or an ancestor of q. Here a blocked start
(q >= 64, a leaf of every older pop's heap) takes H[q] at once and holds its output back; an older pop
that ends at q hands it its value (never larger than the one read, so a pop that has not stopped stays
consistent), and the held output is written once no older hole covers q. A pending pop that would stop
first undoes that write and freezes with every younger pop (younger ones one step longer after its
release); a start needs the youngest pop two levels deep. run() follows the GPU's step semantics (all
reads, then all writes); check() compares with libstdc++'s make_heap + pops (ref_pops).
python tools/pop_spec_sim.py <dump file from PFREF_HEAP_DUMP> [segments]"""
import struct
import sys

import numpy as np


def load(fn, idx):
    b=open(fn,'rb').read(); o=0; i=0
    while o+8<=len(b):
        n,p=struct.unpack_from('ii',b,o)
        if i==idx: return np.frombuffer(b,dtype=np.uint32,count=n,offset=o+8).astype(np.int64), p
        o+=8+4*n; i+=1


def anc(h,q):   # h is q or an ancestor of q
    while q>h: q=(q-1)//2
    return q==h


def ref_pops(keys, npops):
    H=[(k,i) for i,k in enumerate(keys)]; n=len(H)
    # make_heap on keys only (names ride along)
    for x in range((n-2)//2,-1,-1):
        v=H[x]; h=x
        while True:
            c1=2*h+1
            if c1>=n: break
            c=c1
            if c1+1<n and not (H[c1+1][0]<H[c1][0]): c=c1+1
            if H[c][0]<v[0]: break
            H[h]=H[c]; h=c
        H[h]=v
    for i in range(npops):
        q=n-1-i; v=H[q]; H[q]=H[0]; h=0
        while True:
            c1=2*h+1
            if c1>=q: break
            c=c1
            if c1+1<q and not (H[c1+1][0]<H[c1][0]): c=c1+1
            if H[c][0]<v[0]: break
            H[h]=H[c]; h=c
        H[h]=v
    return H


def run(keys, npops, maxpend=1):
    H=[(k+1,i) for i,k in enumerate(keys)]; n=len(H)
    # make_heap (top-down form, same as the reference restatement)
    for x in range((n-2)//2,-1,-1):
        v=H[x]; h=x
        while True:
            c1=2*h+1
            if c1>=n: break
            c=c1
            if c1+1<n and not (H[c1+1][0]<H[c1][0]): c=c1+1
            if H[c][0]<v[0]: break
            H[h]=H[c]; h=c
        H[h]=v
    H += [(0,0),(0,0)] + [(0,0)]*64
    last=n-1; nxt=0
    lanes=[dict(h=None,m=0,v=None,idx=-1) for _ in range(64)]
    pend=[]   # dicts: idx,q,o,old(set of lane ids),stalled,hold
    ff=None; hold_younger=None
    steps=0
    def anc_ok(h,q): return h is not None and anc(h,q)
    while True:
        for sub in (0,1):
            steps+=1
            # deferred writes
            for P in list(pend):
                if not any(anc_ok(lanes[L]['h'],P['q']) for L in P['old'] if lanes[L]['idx']>=0):
                    H[P['q']]=(0,P['o'])
                    pend.remove(P)
                    if P['stalled']: hold_younger=P['idx']   # younger stay frozen this step
            stalled=[P['idx'] for P in pend if P['stalled']]
            ffz=min(stalled) if stalled else None
            # start
            yl=[L for L in lanes if nxt>0 and L['idx']==nxt-1]
            young_ok = not yl or (yl[0]['h'] is not None and yl[0]['h']>=3)   # the youngest pop at depth >= 2
            if sub==0 and nxt<npops and ffz is None and hold_younger is None and young_ok:
                q=last-nxt
                blk=any(L['idx']>=0 and anc_ok(L['h'],q) for L in lanes)
                if not blk or (q>=64 and len(pend)<maxpend):
                    Ln=nxt&63
                    vq=H[q]; r0=H[0]
                    act={i for i,L in enumerate(lanes) if L['idx']>=0}
                    for P in pend: P['old'].discard(Ln)
                    if not blk: H[q]=(0,r0[1])
                    else: pend.append(dict(idx=nxt,q=q,o=r0[1],old=act-{Ln},stalled=False))
                    lanes[Ln]=dict(h=0,m=q,v=vq,idx=nxt)
                    nxt+=1
            # reads
            dec={}
            for i,L in enumerate(lanes):
                if L['idx']<0: continue
                if ffz is not None and L['idx']>=ffz: continue
                if hold_younger is not None and L['idx']>hold_younger: continue
                h=L['h']; c1=2*h+1; m=L['m']
                has=c1<m
                a=H[c1] if has else (0,0); b=H[c1+1] if has else (0,0)
                right=has and c1+1<m and not (b[0]<a[0])
                ch=b if right else a
                stop=(not has) or ch[0]<L['v'][0]
                dec[i]=(h,stop,ch,c1+(1 if right else 0))
            hold_younger=None
            # writes
            ho=[]
            for i,(h,stop,ch,c) in dec.items():
                L=lanes[i]
                isp=[P for P in pend if P['idx']==L['idx']]
                if isp and stop:
                    isp[0]['stalled']=True; continue
                H[h]=L['v'] if stop else ch
                if stop:
                    for P in pend:
                        if h==P['q'] and L['idx']<P['idx']: ho.append((P['idx'],L['v']))
                    lanes[i]=dict(h=None,m=0,v=None,idx=-1)
                else:
                    L['h']=c
            for pidx,v in ho:
                for L in lanes:
                    if L['idx']==pidx: L['v']=v
        if nxt>=npops and all(L['idx']<0 for L in lanes) and not pend: break
        if steps>40*n+1000: raise RuntimeError("stuck at nxt %d pend %s lanes %s"%(nxt,[(P['idx'],P['q'],P['stalled'],sorted(P['old'])) for P in pend],[(L['idx'],L['h'],L['m']) for L in lanes if L['idx']>=0]))
    out=[(x[0]-1 if x[0] else None, x[1]) for x in H[:n]]
    return out, steps

def check(keys, npops, mp):
    R=ref_pops(keys,npops); S,st=run(keys,npops,mp)
    n=len(keys)
    ok=[r[1] for r in R[n-npops:]]==[s[1] for s in S[n-npops:]] and [r[1] for r in R[:n-npops]]==[s[1] for s in S[:n-npops]]
    return ok, st/npops


if __name__ == "__main__":
    fn = sys.argv[1]
    nseg = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    for idx in range(nseg):
        seg = load(fn, idx)
        if seg is None:
            break
        k, p = seg
        k = list(map(int, k))
        p = min(p, len(k) - 1)
        print("segment %d: n %d pops %d  exact %s  steps/pop %.2f" % ((idx, len(k), p) + check(k, p, 1)), flush=True)
