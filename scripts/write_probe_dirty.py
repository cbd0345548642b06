import os, time
MB=1<<20
buf=os.urandom(4*MB)
print(open('/proc/sys/vm/dirty_ratio').read().strip(), open('/proc/sys/vm/dirty_background_ratio').read().strip(), open('/proc/sys/vm/dirty_bytes').read().strip())
for p in ('/sys/fs/cgroup/memory.max','/sys/fs/cgroup/memory.high'):
    try: print(p, open(p).read().strip())
    except Exception as e: print(p, e)
paths=[]
for i in range(16):
    p=f'/tmp/wprobe_{os.getpid()}_{i}'
    fd=os.open(p, os.O_WRONLY|os.O_CREAT|os.O_TRUNC, 0o644)
    t=time.perf_counter()
    for k in range(185): os.write(fd, buf)
    dt=time.perf_counter()-t
    os.close(fd); paths.append(p)
    dirty=[l for l in open('/proc/meminfo') if l.startswith(('Dirty','Writeback:'))]
    print(f"file {i}: {185*4/1024/dt:.2f} GB/s  {' '.join(x.split()[1] for x in dirty)} kB dirty/wb", flush=True)
for p in paths: os.remove(p)
