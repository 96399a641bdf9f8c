"""Resolve the frames of a glog-style crash trace ("@ 0x7f... (unknown)") against a /proc/<pid>/maps dump taken by the
same process (bench.py writes one per leg when BENCH_MAPS is set): library, file offset and the nearest preceding
symbol (dynamic and, when present, static symbol tables via llvm-readelf).  Run on the box that produced the crash
(the libraries must be the same files).

    python3 tools/resolve_frames.py crash.log maps.txt
"""
import bisect
import re
import subprocess
import sys

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def load_maps(path, files_only=True):
    maps = []
    for line in open(path):
        parts = line.split()
        if len(parts) < 5 or (files_only and (len(parts) < 6 or not parts[5].startswith("/"))):
            continue
        lo, hi = (int(x, 16) for x in parts[0].split("-"))
        maps.append((lo, hi, int(parts[2], 16), parts[5] if len(parts) > 5 else "[anon]", parts[1]))
    return sorted(maps)


_syms = {}
_phdrs = {}


def symbols(lib):
    if lib not in _syms:
        out = []
        for flag in ("--dyn-syms", "--symbols"):
            try:
                txt = subprocess.run([READELF, flag, "--wide", "-C", lib], capture_output=True, text=True,
                                     timeout=60).stdout
            except (OSError, subprocess.TimeoutExpired):
                continue
            for ln in txt.splitlines():
                p = ln.split(None, 7)
                if len(p) >= 8 and p[3] == "FUNC" and p[1] != "0000000000000000":
                    out.append((int(p[1], 16), int(p[2]), p[7]))
        out.sort()
        _syms[lib] = out
    return _syms[lib]


def file_to_vaddr(lib, off):
    """File offset -> link-time virtual address through the PT_LOAD program headers."""
    if lib not in _phdrs:
        segs = []
        try:
            txt = subprocess.run([READELF, "-l", "--wide", lib], capture_output=True, text=True, timeout=60).stdout
        except (OSError, subprocess.TimeoutExpired):
            txt = ""
        for ln in txt.splitlines():
            p = ln.split()
            if p and p[0] == "LOAD":
                segs.append((int(p[1], 16), int(p[2], 16), int(p[4], 16)))   # offset, vaddr, filesz
        _phdrs[lib] = segs
    for o, v, sz in _phdrs[lib]:
        if o <= off < o + sz:
            return v + (off - o)
    return off


def main():
    log, maps_path = sys.argv[1], sys.argv[2]
    maps = load_maps(maps_path)
    allm = load_maps(maps_path, files_only=False)
    starts = [m[0] for m in maps]
    addrs = []
    for line in open(log, errors="replace"):
        m = re.search(r"(?:@|PC: @)\s+0x([0-9a-f]+)", line)
        if m:
            addrs.append((line.strip()[:40], int(m.group(1), 16)))
        m = re.search(r"SIGSEGV \(@0x([0-9a-f]+)\)", line)
        if m:
            addrs.append(("fault address", int(m.group(1), 16)))
    for tag, a in addrs:
        i = bisect.bisect_right(starts, a) - 1
        if i < 0 or not (maps[i][0] <= a < maps[i][1]):
            near = [m for m in allm if m[0] <= a < m[1]]
            below = [m for m in allm if m[1] <= a]
            above = [m for m in allm if m[0] > a]
            desc = (f"inside {near[0][3]} {near[0][4]} [{near[0][0]:#x}, {near[0][1]:#x})" if near else
                    "unmapped at dump time; neighbours " +
                    (f"below {below[-1][3]} ends {below[-1][1]:#x}" if below else "") +
                    (f", above {above[0][3]} starts {above[0][0]:#x}" if above else ""))
            print(f"{a:#x}  [not in a file mapping: {desc}]  {tag}")
            continue
        lo, hi, off, lib, _ = maps[i]
        fo = a - lo + off
        va = file_to_vaddr(lib, fo)
        name = "?"
        syms = symbols(lib)
        j = bisect.bisect_right([s[0] for s in syms], va) - 1
        if j >= 0:
            s = syms[j]
            name = f"{s[2]}+{va - s[0]:#x}" + ("" if va < s[0] + max(s[1], 1) else " (past symbol end)")
        print(f"{a:#x}  {lib.split('/')[-1]}+{fo:#x}  {name}")


if __name__ == "__main__":
    main()
