"""Instruction mix of one kernel in a gfx950 assembly listing (hipcc -S --offload-device-only).

usage: python tools/isa_stats.py <file.s> <kernel-name-substring>
"""
import sys
from collections import Counter


def main():
    s = open(sys.argv[1]).read()
    sub = sys.argv[2]
    names = [l.split(':')[0] for l in s.split('\n') if sub in l and l.split(":")[0] and not l.startswith((".", "\t", ";")) and ":" in l]
    for name in names:
        i = s.index(name + ':')
        j = s.index('.Lfunc_end', i)
        ins = [l.strip() for l in s[i:j].split('\n') if l.startswith('\t') and not l.strip().startswith(('.', ';'))]
        c = Counter()
        for l in ins:
            op = l.split()[0]
            c['valu' if op.startswith('v_') else 'salu' if op.startswith('s_') else
              'vmem' if op.startswith(('global_', 'buffer_', 'flat_')) else op] += 1
        print(name[:90], len(ins), dict(c))
        if len(sys.argv) > 3:
            for op, k in Counter(l.split()[0] for l in ins).most_common(int(sys.argv[3])):
                print(f"   {op:28s} {k}")


if __name__ == "__main__":
    main()
