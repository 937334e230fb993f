#!/usr/bin/env python3
"""Which host (CPU / RAM) energy sources this machine exposes to an unprivileged process: amd-smi CPU sockets
(HSMP), RAPL powercap zones, hwmon energy sensors; plus the CPU model and socket count the TDP model uses."""
import glob
import os

def rd(p):
    try:
        with open(p) as fh:
            return fh.read().strip()
    except Exception as e:  # noqa: BLE001
        return f"ERR {type(e).__name__}: {e}"

print("uid", os.getuid())
models = sorted({l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")})
phys = sorted({l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("physical id")})
print("cpu models", models, "sockets", len(phys), "logical cpus", os.cpu_count())
print("meminfo", rd("/proc/meminfo").splitlines()[:2])
for z in sorted(glob.glob("/sys/class/powercap/*")):
    print("powercap", z, rd(z + "/name"), rd(z + "/energy_uj"), rd(z + "/max_energy_range_uj"))
for h in sorted(glob.glob("/sys/class/hwmon/hwmon*")):
    nm = rd(h + "/name")
    ens = sorted(glob.glob(h + "/energy*_input"))[:4]
    pws = sorted(glob.glob(h + "/power*_input"))[:4]
    print("hwmon", h, nm, [(os.path.basename(e), rd(e)) for e in ens], [(os.path.basename(p), rd(p)) for p in pws])
print("hsmp dev", glob.glob("/dev/hsmp*"), "msr", os.path.exists("/dev/cpu/0/msr"))
try:
    import amdsmi
    try:
        amdsmi.amdsmi_init(amdsmi.AmdSmiInitFlags.INIT_AMD_CPUS)
        cs = amdsmi.amdsmi_get_cpusocket_handles()
        print("amdsmi cpu sockets", len(cs))
        for c in cs:
            print("  energy", amdsmi.amdsmi_get_cpu_socket_energy(c), "power", amdsmi.amdsmi_get_cpu_socket_power(c))
        amdsmi.amdsmi_shut_down()
    except Exception as e:  # noqa: BLE001
        print("amdsmi cpu init ERR", repr(e))
except Exception as e:  # noqa: BLE001
    print("amdsmi import ERR", e)
