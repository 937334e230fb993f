set -x
id; nproc; free -g | head -2
timeout -k 10 120 python - <<'PY'
import time, torch
print(torch.__version__, torch.cuda.is_available(), torch.cuda.device_count())
p = torch.cuda.get_device_properties(0); print(p)
try:
    import amdsmi
    amdsmi.amdsmi_init()
    hs = amdsmi.amdsmi_get_processor_handles()
    print("handles", len(hs))
    h = hs[0]
    for fn in ["amdsmi_get_energy_count","amdsmi_get_power_info","amdsmi_get_gpu_activity","amdsmi_get_gpu_metrics_info"]:
        try:
            r = getattr(amdsmi, fn)(h); 
            if fn=="amdsmi_get_gpu_metrics_info":
                r = {k:v for k,v in r.items() if any(s in k for s in ["energy","power","activity","timestamp"])}
            print(fn, r)
        except Exception as e: print(fn, "ERR", e)
    e0 = amdsmi.amdsmi_get_energy_count(h)
    x = torch.randn(8192,8192,device="cuda",dtype=torch.bfloat16)
    torch.cuda.synchronize(); t=time.time()
    for _ in range(200): y = x@x
    torch.cuda.synchronize(); dt=time.time()-t
    e1 = amdsmi.amdsmi_get_energy_count(h)
    print("dt", dt, "e0", e0, "e1", e1)
    for i in range(20):
        print(time.time(), amdsmi.amdsmi_get_energy_count(h)); time.sleep(0.01)
    try:
        cs = amdsmi.amdsmi_get_cpusocket_handles(); print("cpusockets", len(cs))
        print(amdsmi.amdsmi_get_cpu_socket_energy(cs[0]))
    except Exception as e: print("cpu ERR", e)
except Exception as e:
    import traceback; traceback.print_exc()
PY
ls /sys/class/powercap/ 2>&1 | head; cat /sys/class/powercap/intel-rapl:0/energy_uj 2>&1; ls /sys/class/hwmon/ | head; for h in /sys/class/hwmon/hwmon*; do echo $h $(cat $h/name); done 2>&1 | head -40
rocm-smi --showpower --showenergycounter 2>&1 | head -30
amd-smi metric -p -E 2>&1 | head -40
