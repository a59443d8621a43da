"""Memory-op / wait / branch skeleton of one kernel in a hipcc -S device assembly file, to spot
loads whose results are waited for before independent loads are issued:
    python tools/isa_loads.py <file.s> <substring of the kernel symbol> [max lines]"""
import sys


def main(path, sub, limit=400):
    s = open(path).read()
    i = next(k for k in range(len(s)) if s.startswith('_Z', k) and sub in s[k:s.index('\n', k)]
             and s[k:s.index('\n', k)].split(';')[0].strip().endswith(':'))
    j = s.index('.Lfunc_end', i)
    n = 0
    for ln, l in enumerate(s[i:j].split('\n')):
        t = l.strip()
        if t.startswith(('global_load', 'global_store', 's_waitcnt', 's_cbranch', 'buffer_', 'global_atomic',
                         's_load', 'ds_')) or (t.startswith('.LBB') and t.endswith(':')):
            print(ln, t)
            n += 1
            if n >= limit:
                break


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], *(int(a) for a in sys.argv[3:4]))
