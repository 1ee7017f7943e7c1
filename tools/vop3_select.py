import re, sys
INLINE_F = {"0.5", "-0.5", "1.0", "-1.0", "2.0", "-2.0", "4.0", "-4.0", "0.15915494"}
def inline(x):
    if re.fullmatch(r"-?\d+", x): return -16 <= int(x) <= 64
    return x in INLINE_F
pat = re.compile(r"^(\s*)v_cndmask_b32_e32 (v\d+), ([^,]+), (v\d+), vcc(\s*;.*)?$")
n = skipped = 0
out = []
for line in open(sys.argv[1]):
    m = pat.match(line.rstrip("\n"))
    if m:
        ind, d, s0, s1, _ = m.groups()
        if re.fullmatch(r"v\d+", s0) or inline(s0):
            line = f"{ind}v_cndmask_b32_e64 {d}, {s0}, {s1}, vcc\n"; n += 1
        else:
            skipped += 1
    out.append(line)
open(sys.argv[2], "w").writelines(out)
print("rewrote", n, "skipped", skipped, file=sys.stderr)
