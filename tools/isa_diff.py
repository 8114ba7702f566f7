"""Compare the gfx950 instructions of kernels between two device-assembly dumps.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
          --offload-device-only -S gp_round.hip -o before.s
    ... edit ...
    python tools/isa_diff.py before.s after.s [kernel-substring ...]

For every kernel whose mangled name contains one of the substrings (default: every
kernel in the first file), the body between its label and `.Lfunc_end` is compared
after dropping comments, blank lines and basic-block label names (so a renumbered
label is not a difference).  Prints one line per kernel and exits 1 on any
difference.  Used to show that a source clean-up left a kernel's code unchanged.
"""
import re
import sys


def bodies(path):
    out, cur, name = {}, None, None
    label = re.compile(r"^(_Z\w+):")
    with open(path) as f:
        for line in f:
            m = label.match(line)
            if m and name is None:
                name, cur = m.group(1), []
                continue
            if name is not None:
                if line.startswith(".Lfunc_end"):
                    out[name] = cur
                    name = None
                    continue
                s = line.split(";", 1)[0].strip()
                if not s or s.startswith(".loc") or s.startswith(".cfi"):
                    continue
                s = re.sub(r"\.LBB\d+_\d+", ".LBB", s)
                s = re.sub(r"\.Ltmp\d+", ".Ltmp", s)
                cur.append(s)
    return out


def main():
    a, b = bodies(sys.argv[1]), bodies(sys.argv[2])
    keys = sys.argv[3:]
    names = [n for n in a if not keys or any(k in n for k in keys)]
    bad = 0
    for n in names:
        if n not in b:
            print(f"MISSING {n}")
            bad += 1
            continue
        ia = [s for s in a[n] if not s.startswith(".")]
        ib = [s for s in b[n] if not s.startswith(".")]
        same = ia == ib
        bad += not same
        print(f"{'same' if same else 'DIFF'} {n}: {len(ia)} / {len(ib)} instructions")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
