"""Names the frames of a stripped ROCm library's backtrace (round 5).

    python3 tools/symbolize_frames.py <lib.so> <offset> [<offset> ...]

libamdhip64 / libhsa-runtime64 ship without symbols, so for each offset this
finds the enclosing function from the .eh_frame FDE ranges (readelf -wf),
disassembles it (objdump) and prints the read-only strings it references
(log formats, source file names) and the exported functions it calls.  The
strings name the CLR / ROCr function (e.g. "Deleting hardware queue %p with
refCount 0" is roc::Device::releaseQueue).  The output for
profiles/r04_procs_exit_stall.txt is profiles/r05_exit_stall_symbolized.txt.
"""
import subprocess,re,sys,bisect
lib=sys.argv[1]; addrs=[int(a,16) for a in sys.argv[2:]]
fr=subprocess.run(['readelf','-wf',lib],capture_output=True,text=True).stdout
rng=[(int(a,16),int(b,16)) for a,b in re.findall(r'FDE cie=\w+ pc=([0-9a-f]+)\.\.([0-9a-f]+)',fr)]
rng.sort()
data=open(lib,'rb').read()
# section map for file offsets
secs=subprocess.run(['readelf','-S','-W',lib],capture_output=True,text=True).stdout
smap=[]
for m in re.finditer(r'\]\s+(\S+)\s+\S+\s+([0-9a-f]+)\s+([0-9a-f]+)\s+([0-9a-f]+)',secs):
    smap.append((int(m.group(2),16),int(m.group(3),16),int(m.group(4),16),m.group(1)))
def rd(va):
    for a,o,s,n in smap:
        if a<=va<a+s and a:
            off=o+va-a; e=data.find(b'\0',off,off+200)
            try: return data[off:e].decode()
            except: return None
syms={}
for l in subprocess.run(['nm','-D','--defined-only',lib],capture_output=True,text=True).stdout.split('\n'):
    p=l.split()
    if len(p)>=3: syms[int(p[0],16)]=p[2]
for a in addrs:
    f=[r for r in rng if r[0]<=a<r[1]]
    if not f: print(hex(a),'no fde'); continue
    lo,hi=f[0]
    dis=subprocess.run(['objdump','-d','--no-show-raw-insn',f'--start-address={lo}',f'--stop-address={hi}',lib],capture_output=True,text=True).stdout
    strs=[];calls=[]
    for m in re.finditer(r'#\s*([0-9a-f]+)',dis):
        s=rd(int(m.group(1),16))
        if s and len(s)>3 and s.isprintable(): strs.append(s)
    for m in re.finditer(r'call\s+([0-9a-f]+)\s*<([^>]+)>',dis): calls.append(m.group(2))
    print(f'== {hex(a)} in fn {hex(lo)}..{hex(hi)} ({syms.get(lo,"")}) size {hi-lo}')
    for s in dict.fromkeys(strs): print('   str:',s[:120])
    print('   calls:',sorted(set(c for c in calls if '@' in c))[:25])
