set -e
mkdir -p gpurun_out/occ
for W in 1 2; do for L in 2 6 9 12; do
SF_TRACE_WAVES=$W SF_LEVELS=$L timeout -k 10 60 python scripts/tile_schedule.py --reps 1 --out gpurun_out/occ/w${W}_l${L}.npy > gpurun_out/occ/w${W}_l${L}.txt 2>&1
done; done
python3 - <<'PY'
import numpy as np
for W in (1,2):
  for L in (2,6,9,12):
    tr=np.load(f"gpurun_out/occ/w{W}_l{L}.npy").astype(np.int64)
    s,e,hw=tr[:,0],tr[:,1],tr[:,2]; xcc=hw>>32; h=hw&0xffffffff
    wave=h&0xf; simd=(h>>4)&3; cu=(h>>8)&0xf; sh=(h>>12)&1; se=(h>>13)&7
    cuid=((xcc*8+se)*2+sh)*16+cu
    best=0
    for q in (10,20,30,40,50):
        t=np.percentile(s,q); live=(s<=t)&(e>t); c=np.bincount(cuid[live]); best=max(best,c.max())
    lds=(16+(L-1)*176)*4
    print(f"W={W} L={L} lds/wave={lds} slots={wave.max()+1} maxlive/CU={best} span={(e.max()-s.min())/100:.0f}us")
PY
