import numpy as np
rng=np.random.default_rng(0)
cap=1<<18; n=cap//2
for B in (1,2,4,8):
    h=rng.integers(0,cap//B,size=n)*B
    table=-np.ones(cap,np.int64); pos=np.zeros(n,np.int64)
    for i,s in enumerate(h):
        while table[s]>=0: s=(s+1)%cap
        table[s]=i; pos[i]=s
    disp=(pos-h)%cap
    rounds=disp//B+1
    q=rng.integers(0,n,size=64*4096)
    w=rounds[q].reshape(-1,64).max(1)
    print(B, "mean disp", disp.mean().round(2), "lane rounds", rounds.mean().round(3), "wave rounds mean", w.mean().round(2), "p99", np.percentile(w,99))
