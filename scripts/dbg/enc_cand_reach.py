"""CPU study (round 6): how far back the encoder's candidates lie.  For each
64-lane window of the one-wave encoder's parse (lzo1x_encode_fast.hip; the
sequential LZO1X-1 parse of SURVEY.md Appendix A.1 on ITB blocks, windows capped
at 6 matches, conflicts ignored), the largest candidate distance of all lanes and
of the path lanes: the share of windows an LDS ring of the last R input bytes
would serve without a global candidate read.  Usage: python scripts/dbg/enc_cand_reach.py"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pomegranate_amd import synth
K=16384
def prim(b,p):
    v=((((b[p+3]<<6)^b[p+2])<<5)^b[p+1]); v=(v<<5)^b[p]
    return ((v*33)>>5)&(K-1)
def sec(h): return (h&0x7FF)^0x201F
def sim(b, reaches=(1024,2048,3584,8192,16384)):
    n=len(b); d=[0]*K; ip=4; ip_end=n-13
    # sequential parse, recording per position the decision; windows emulate the kernel's 64-lane/6-match cut
    nwin=0; allnear={r:0 for r in reaches}; lanes_far={r:0 for r in reaches}; lanes=0
    pathnear={r:0 for r in reaches}
    while ip<ip_end:
        nwin+=1
        # pre-window probe of all lanes
        dist=[]
        for l in range(64):
            p=ip+l
            if p>=ip_end: break
            h1=prim(b,p); c=d[h1]; ds=[]
            if c and p-(c-1)<=0xBFFF:
                cc=c-1; ds.append(p-cc)
                if not (p-cc<=0x800 or b[cc+3]==b[p+3]):
                    c2=d[sec(h1)]
                    if c2 and p-(c2-1)<=0xBFFF: ds.append(p-(c2-1))
            dist.append(max(ds) if ds else 0)
        lanes+=len(dist)
        # now advance the real parse through the window (64 lanes, 6 matches)
        q=ip; nm=0; pathd=[]
        while q<ip+64 and q<ip_end and nm<6:
            h1=prim(b,q); slot=h1; c=d[h1]; ok=False
            if c and q-(c-1)<=0xBFFF:
                cc=c-1
                if q-cc<=0x800 or b[cc+3]==b[q+3]: ok=True
                else:
                    slot=sec(h1); c=d[slot]
                    if c and q-(c-1)<=0xBFFF:
                        cc=c-1
                        if q-cc<=0x800 or b[cc+3]==b[q+3]: ok=True
            if ok and not (b[cc]==b[q] and b[cc+1]==b[q+1] and b[cc+2]==b[q+2]): ok=False
            d[slot]=q+1
            if ok:
                pathd.append(q-cc)
                L=3
                while q+L<n and b[cc+L]==b[q+L]: L+=1
                q+=L; nm+=1
            else:
                q+=1
        for r in reaches:
            if max(dist, default=0)<=r: allnear[r]+=1
            if max(pathd, default=0)<=r: pathnear[r]+=1
            lanes_far[r]+=sum(1 for x in dist if x>r)
        ip=q
    return nwin, allnear, pathnear, lanes_far, lanes
a,offs,lens=synth.batch(synth.ITB,0,[65536]*4)
for i in range(4):
    b=a[int(offs[i]):int(offs[i])+65536].tobytes()
    nw,an,pn,lf,la=sim(b)
    print(i,"windows",nw,"all-lanes-near",{r:round(v/nw,2) for r,v in an.items()},"path-near",{r:round(v/nw,2) for r,v in pn.items()},"far-lane frac",{r:round(v/la,3) for r,v in lf.items()})
