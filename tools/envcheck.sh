for f in /proc/sys/kernel/numa_balancing /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag /proc/sys/vm/zone_reclaim_mode; do echo "$f: $(cat $f 2>&1)"; done
ls /sys/devices/system/node/ | grep node; for n in /sys/devices/system/node/node*; do echo "$n $(cat $n/cpulist)"; done
grep Cpus_allowed_list /proc/self/status; nproc
for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.stat /sys/fs/cgroup/memory.max; do echo "$f:"; cat $f 2>&1; done
