import re,sys,subprocess
src=sys.argv[1]
r=subprocess.run(["/opt/rocm/bin/hipcc","-O3","-fPIC","-std=c++17","--offload-arch=gfx950","-I","kdl/csrc","-x","hip","-c",src,"-o","/tmp/x.o","-Rpass-analysis=kernel-resource-usage"],capture_output=True,text=True)
cur=None; rows={}
for l in r.stderr.splitlines():
    m=re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]): (\S+)",l)
    if not m: continue
    k,v=m.groups()
    if k=="Function Name": cur=v; rows[cur]={}
    else: rows[cur][k]=v
flt=sys.argv[2] if len(sys.argv)>2 else ""
for f,d in rows.items():
    if flt in f: print(f[-60:], d.get("VGPRs"), d.get("AGPRs"), "spill", d.get("VGPRs Spill"), "occ", d.get("Occupancy [waves/SIMD]"))
