"""Per-block offsets of the dataflow Cholesky's critical chain from a CVXG_DF_TRACE file (k_dataflow.hip marks), in us from
POTRF(k) start: POTRF(k) done, block k+1's staging begin / staged / slice 2 done / last L^-1 row-block in hand / slices done,
POTRF(k+1) start, the fix hook of POTRF(k+1); then the worker tasks feeding block row k+1 (claim / ready / done)."""
import sys, numpy as np
raw=open(sys.argv[1],'rb').read()
nq,nb=(int(v) for v in np.frombuffer(raw[:8],dtype=np.int32))
R=((len(raw)-8-4*nq)//32-nq)//nb  # chain records per block (k_dataflow.hip: 5 since round 5, 3 before)
tr=np.frombuffer(raw[8+4*nq:8+4*nq+32*(nq+R*nb)],dtype=np.uint64).reshape(nq+R*nb,4).astype(np.int64)
ch=tr[nq:].reshape(nb,R,4)
us=lambda v:v/100.0
rows=[]
for k in range(2,nb-2):
    A=ch[k,0,0]; B=ch[k,0,2]
    stg0=ch[k,1,0]; C=ch[k,1,1]; D=ch[k,1,3]; E=ch[k,1,2]
    F=ch[k+1,0,0]
    fix0=ch[k,2,0]; fix1=ch[k,2,1]; fix2=ch[k,2,2]  # fix of block k+1 (waits POTRF(k) done)
    s2=ch[k+1,0,1]
    b2in=ch[k,2,3]; b2done=ch[k,0,3]  # chain-owned b-2 staging (k_dataflow.hip own_b2): inputs in / panel applied
    rbp=[ch[k,3,i] if R>3 else 0 for i in range(4)]  # POTRF(k)'s L^-1 row-block flags raised (wave 3)
    bat=[ch[k,4,i] if R>4 else 0 for i in range(3)]  # the batch of block k+1: loads landed, TRSM products, updates
    rows.append([us(B-A),us(stg0-A),us(C-A),us(s2-A) if s2>A else np.nan,us(D-A) if D>A else np.nan,us(E-A),us(F-A),us(fix0-F) if fix0>0 else 0, us(fix1-F) if fix1>0 else 0,us(fix2-F) if fix2>0 else 0,
                 us(b2in-A) if b2in>0 else np.nan, us(b2done-A) if b2done>0 else np.nan]+[us(v-A) if v>0 else np.nan for v in rbp]+[us(v-A) if v>0 else np.nan for v in bat])
r=np.array(rows)
# (round 6: record 4 = the forward-substitution slices: packages 0..2 in LDS, slice 0 done, slice 1 done; 'lastrow' =
# package 3 in LDS)
names=['potrf_done','stage_begin(k+1)','staged(k+1)','slice2done(k+1)','pkg3_in(k+1)','slices_done(k+1)','potrf_start(k+1)','fix0(k+1)-F','fix1-F','fix2-F','b2_inputs(k+1)','b2_applied(k+1)','rb0_flag(k)','rb1_flag(k)','rb2_flag(k)','rb3_flag(k)','pkg012_in(k+1)','slice0_done(k+1)','slice1_done(k+1)']
for i,nm in enumerate(names):
    print(f"{nm:22s} mean {np.nanmean(r[:,i]):7.2f} med {np.nanmedian(r[:,i]):7.2f} min {np.nanmin(r[:,i]):7.2f} max {np.nanmax(r[:,i]):7.2f}")
order=np.frombuffer(raw[8:8+4*nq],dtype=np.uint32)
typ,kk,ii,jj=order>>30,(order>>20)&1023,(order>>10)&1023,order&1023
rec={(int(typ[x]),int(ii[x]),int(jj[x]),int(kk[x])):tr[x] for x in range(nq)}
res=[]
for k in range(2,nb-2):
    s0=ch[k,0,0]
    row=[]
    for key in ((1,k+1,k-1,k-1),(2,k+1,k,k-1),(2,k+1,k+1,k-1),(1,k+1,k-2,k-2),(2,k+1,k,k-2),(2,k+1,k+1,k-2)):
        r=rec.get(key)
        row += [np.nan]*3 if r is None else [(v-s0)/100.0 for v in r[:3]]
    row.append((ch[k,1,1]-s0)/100.0)
    res.append(row)
res=np.array(res)
lab=['TRSM(k+1,k-1)','UPD(k+1,k,k-1)','UPD(k+1,k+1,k-1)','TRSM(k+1,k-2)','UPD(k+1,k,k-2)','UPD(k+1,k+1,k-2)']
for i,l in enumerate(lab):
    c=res[:,3*i:3*i+3]
    ok=~np.isnan(c[:,0])
    if ok.sum()==0: print(l,'none'); continue
    print(f"{l:18s} n={ok.sum():3d} claim {np.nanmedian(c[:,0]):7.2f} ready {np.nanmedian(c[:,1]):7.2f} done {np.nanmedian(c[:,2]):7.2f}  (medians, us rel POTRF(k) start)")
print('staged', np.median(res[:,-1]))
# which is last before staging?
# the chain's own panel work on block row k+1 (TRSM(k+1,k-1), UPDATE(k+1,k+1,k-1), UPDATE(k+1,k,k-1)), when stamped
if R >= 5 and ch[2:nb-2, 3, 0].min() > 0:
    lab = ['inputs ready', 'loads landed', 'L_k+1,k-1 published', 'L_k,k-1 in LDS', 'updates done']
    vals = []
    for k in range(2, nb - 2):
        A = ch[k, 0, 0]
        vals.append([(ch[k, 3, f] - A) / 100.0 for f in range(4)] + [(ch[k, 4, 0] - A) / 100.0])
    vals = np.array(vals)
    for i, l in enumerate(lab):
        print(f"panel {l:22s} med {np.median(vals[:, i]):7.2f} mean {vals[:, i].mean():7.2f}")
# L^-1 row-block hand-offs: flags raised by POTRF(k)'s waves (record 5), the consumer's batch / wait for the last one
if R >= 6 and ch[2:nb-2, 5, 3].min() > 0:
    v = np.array([[(ch[k, 5, f] - ch[k, 0, 0]) / 100.0 for f in range(4)] for k in range(2, nb - 2)])
    for f in range(4):
        print(f"rb{f} flag raised        med {np.median(v[:, f]):7.2f} mean {v[:, f].mean():7.2f}")
    nbat = ch[2:nb-2, 4, 3]
    print("batch sizes", {int(x): int((nbat == x).sum()) for x in np.unique(nbat)})
    bd = np.array([(ch[k, 4, 2] - ch[k, 0, 0]) / 100.0 for k in range(2, nb - 2)])
    print(f"batch done             med {np.median(bd):7.2f} mean {bd.mean():7.2f}")
    w = [(ch[k, 4, 1] - ch[k, 0, 0]) / 100.0 for k in range(2, nb - 2) if ch[k, 4, 1] > ch[k, 0, 0]]
    if w:
        print(f"wait for rb3 begins    med {np.median(w):7.2f} mean {np.mean(w):7.2f} (n={len(w)})")
