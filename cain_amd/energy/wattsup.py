"""Watts up? Pro external wall-power meter logger.

Reference: experiment-runner/Plugins/Profilers/WattsUpPro.py:5-73 (pyserial,
115200 baud, ``#L,W,3,<mode>,,<interval>;`` logging command, ``#d,...`` data
frames with W/V/A at fields 3/4/5 in tenths / tenths / thousandths).

pyserial is not part of this image, so the port is driven with ``termios``
directly (any object with ``readline``/``write`` can be injected for tests).
The reference's latent ``str``-to-serial bug in ``mode(INTERNAL_MODE)`` is fixed.
"""
from __future__ import annotations

import datetime
import os
import platform
import time
from dataclasses import dataclass
from typing import List, Optional


@dataclass
class WattsUpSample:
    t: float
    watts: float
    volts: float
    amps: float


def parse_frame(line: bytes) -> Optional[WattsUpSample]:
    if not line.startswith(b"#d"):
        return None
    fields = line.strip().rstrip(b";").split(b",")
    if len(fields) <= 5:
        return None
    try:
        return WattsUpSample(time.time(), float(fields[3]) / 10, float(fields[4]) / 10, float(fields[5]) / 1000)
    except ValueError:
        return None


class _TermiosPort:
    def __init__(self, path: str, baud: int = 115200):
        import termios
        import tty

        self.fd = os.open(path, os.O_RDWR | os.O_NOCTTY)
        tty.setraw(self.fd)
        attrs = termios.tcgetattr(self.fd)
        speed = getattr(termios, f"B{baud}")
        attrs[4] = attrs[5] = speed
        termios.tcsetattr(self.fd, termios.TCSANOW, attrs)
        self._buf = b""

    def write(self, data: bytes) -> None:
        os.write(self.fd, data)

    def readline(self) -> bytes:
        while b"\n" not in self._buf:
            chunk = os.read(self.fd, 256)
            if not chunk:
                break
            self._buf += chunk
        line, sep, rest = self._buf.partition(b"\n")
        self._buf = rest
        return line + sep

    def close(self) -> None:
        os.close(self.fd)


class WattsUpPro:
    EXTERNAL_MODE = "E"
    INTERNAL_MODE = "I"
    TCPIP_MODE = "T"
    FULLHANDLING = 2

    def __init__(self, port: Optional[str] = None, interval: float = 1.0, serial_port=None):
        if serial_port is None:
            if port is None:
                port = "/dev/tty.usbserial-A1000wT3" if platform.system() == "Darwin" else "/dev/ttyUSB0"
            if not os.path.exists(port):
                raise RuntimeError(f"Invalid port: serial port {port} does not exist")
            serial_port = _TermiosPort(port)
        self.s = serial_port
        self.interval = interval
        self.samples: List[WattsUpSample] = []

    def mode(self, runmode: str) -> None:
        self.s.write(("#L,W,3,%s,,%d;" % (runmode, self.interval)).encode())
        if runmode == self.INTERNAL_MODE:
            self.s.write(("#O,W,1,%d" % self.FULLHANDLING).encode())

    def log(self, timeout: float, logfile: Optional[str] = None) -> List[WattsUpSample]:
        self.mode(self.EXTERNAL_MODE)
        out = open(logfile, "w") if logfile else None
        n = 0
        t_end = time.time() + timeout
        try:
            while time.time() < t_end:
                s = parse_frame(self.s.readline())
                if s is None:
                    continue
                self.samples.append(s)
                if out:
                    out.write("%s %d %3.1f %3.1f %5.3f\n" % (datetime.datetime.now(), n, s.watts, s.volts, s.amps))
                n += self.interval
        finally:
            if out:
                out.close()
        return self.samples

    def energy_j(self) -> float:
        """Trapezoidal integral of the logged power."""
        s = self.samples
        return sum((b.t - a.t) * (a.watts + b.watts) / 2 for a, b in zip(s, s[1:]))
