"""Instruction mix of each loop (label .. backward branch) in a kernel's ISA listing.
usage: python tools/loopstat.py file.s kernel_substring"""
import re, sys, collections
lines = open(sys.argv[1]).read().split("\n")
name = sys.argv[2]
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % name, l))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
body = lines[start:end + 1]
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\S+:", l)}
for i, l in enumerate(body):
    m = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\.LBB\S+)", l)
    if m and m.group(2) in labels and labels[m.group(2)] < i:
        seg = body[labels[m.group(2)]:i + 1]
        ins = [x.split()[0] for x in seg if x.startswith("\t") and not x.strip().startswith((";", "."))]
        c = collections.Counter(ins)
        print(f"loop {m.group(2)} .. line {i}: {len(ins)} instrs")
        print("   ", ", ".join(f"{k}:{v}" for k, v in c.most_common(14)))
