"""CPU study (round 6): executor steps per 64 KiB ITB block when each window's
ops (64) run by dependency level instead of in batches, after R forwarding rounds
(the decoder's rule, lzo1x_decode_fast.hip); windows with more than WMAX bytes of
output keep the batch rule.  Extends scripts/dbg/dec_level_sim.py (its parse and
compressor).  Usage: python scripts/dbg/dec_level_study.py"""
import sys, bisect, collections
import os
_sim = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dec_level_sim.py")
sys.argv = [sys.argv[0]]
__file__ = _sim
exec(open(_sim).read().split("tb = tl = tw = tlev = 0")[0])
# within-window (64 ops) forwarding with R rounds over the window only (sources before the window final),
# then either batches (current rule) or levels; windows whose output exceeds WMAX use batches.
def win(w, R, mode, WMAX):
    n=len(w); o=[x[0] for x in w]; L=[x[1] for x in w]
    kind=["lit" if x[2]==0 else "out" for x in w]
    db=[0 if x[2]==0 else x[0]-x[2] for x in w]
    dp=[0 if x[2]==0 or x[2]>=x[1] else x[2] for x in w]
    o0=o[0]
    for _ in range(R):
        nd=list(db); nk=list(kind); ch=0
        for i in range(n):
            if kind[i]!="out": continue
            span=dp[i] or L[i]
            if db[i]+span<=o0: continue
            k=bisect.bisect_right(o, db[i])-1
            if k<0 or k>=i: continue
            r=db[i]-o[k]
            if kind[k]=="lit":
                if db[i]+span<=o[k]+L[k]: nd[i]=db[k]+r; nk[i]="lit"; ch+=1
                continue
            if dp[k]: r%=dp[k]
            if db[i]+span<=o[k]+L[k] and (not dp[k] or r+span<=dp[k]):
                if db[k]+r!=db[i] or kind[k]!=kind[i]: nd[i]=db[k]+r; nk[i]=kind[k]; ch+=1
        db=nd; kind=nk
        if not ch: break
    chunks=[(x+15)//16 for x in L]
    wtot=sum(L)
    if mode=="batch" or wtot>WMAX:
        send=[0 if kind[i]!="out" else db[i]+(dp[i] or L[i]) for i in range(n)]
        steps=0; s=0
        while s<n:
            e=next((i for i in range(s+1,n) if kind[i]=="out" and send[i]>o[s]), n)
            steps+=-(-sum(chunks[s:e])//64); s=e
        return steps, wtot>WMAX
    lev=[0]*n
    for i in range(n):
        if kind[i]!="out": continue
        lo=db[i]; hi=db[i]+(dp[i] or L[i])
        if hi<=o0: continue
        k=bisect.bisect_right(o, hi-1)-1; m=-1
        while k>=0 and o[k]+L[k]>lo: m=max(m,lev[k]); k-=1
        lev[i]=m+1
    h=collections.Counter()
    for i in range(n): h[lev[i]]+=chunks[i]
    return sum(-(-c//64) for c in h.values()), False

B=16
for mode,R,WMAX in (("batch",3,0),("level",3,3072),("level",4,3072),("level",6,3072),("level",8,3072),("level",8,2048),("level",8,4096)):
    tot=0; big=0; nw=0
    for b in range(B):
        data=synth.block(synth.ITB, 4242+b, 65536)
        ops=ops_of(compress(data))
        for w0 in range(0,len(ops),64):
            s,bg=win(ops[w0:w0+64],R,mode,WMAX); tot+=s; big+=bg; nw+=1
    print(f"{mode} R={R} WMAX={WMAX}: steps/block {tot/B:.1f}, windows/block {nw/B:.1f}, batch-mode windows {big/nw:.2%}")
