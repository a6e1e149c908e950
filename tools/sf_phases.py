"""Summarise sf_kernel's per-wavefront phase clocks (timing build -DNMPC_SF_TIMING, env NMPC_SF_CYCLES=<file>).

Each launch appends [waves][8] uint64: wall-clock ticks (100 MHz) at the wavefront's start, after the table copy,
after the backward sweep, after the forward sweep, then the shader cycles at the same points. Usage:
    python tools/sf_phases.py <file> <batch> <instances per wave>
Prints, for the last launch in the file: the spread of start times (dispatch), and per phase the median / p90 /
max duration in microseconds and cycles, and the launch's span."""
import sys

import numpy as np


def main():
    path, B, ipw = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    raw = np.fromfile(path, dtype=np.uint64)
    n = (B + 3) // 4 * 8 * 2                          # words per launch (the host's allocation)
    last = raw[-n:].reshape(-1, 8)[: (B + ipw - 1) // ipw].astype(np.int64)
    w, c = last[:, :4], last[:, 4:]
    t0 = w[:, 0].min()
    print(f"launches in file: {raw.size // n}; waves {len(w)}")
    print(f"start spread: p50 {np.median(w[:, 0] - t0) / 100:.2f} us, max {(w[:, 0] - t0).max() / 100:.2f} us; "
          f"span {(w[:, 3].max() - t0) / 100:.2f} us")
    for i, name in enumerate(("table copy", "backward", "forward")):
        dw = (w[:, i + 1] - w[:, i]) / 100.0
        dc = c[:, i + 1] - c[:, i]
        print(f"{name:11s}: {np.median(dw):7.2f} / {np.percentile(dw, 90):7.2f} / {dw.max():7.2f} us   "
              f"{np.median(dc):9.0f} / {np.percentile(dc, 90):9.0f} cycles")


if __name__ == "__main__":
    main()
