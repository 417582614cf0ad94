"""Per-layer comparison of two bench layer dumps (PPS_BENCH_LAYERS):
  python scripts/layer_ab.py A.json B.json  -> us per launch, ratio B/A, TF"""
import json
import sys

H2 = 0x800


def main():
    a, b = (json.load(open(p)) for p in sys.argv[1:3])
    print('%-42s %8s %8s %6s %6s %6s %7s' % ('layer', 'A us', 'B us', 'B/A', 'tileA', 'tileB',
                                            'B TF'))
    ta = tb = 0.0
    for k in list(a) + [k for k in b if k not in a]:
        x, y = a.get(k), b.get(k)
        if (x and not x['gemm']) or (y and not y['gemm']):
            continue
        xa = x['ms'] * 1e3 if x else 0.0
        yb = y['ms'] * 1e3 if y else 0.0
        ta += xa
        tb += yb
        print('%-42s %8.1f %8.1f %6s %6s %6s %7s' % (
            k[:42], xa, yb, '%.2f' % (yb / xa) if x and y else '-',
            '%x' % x['tile'] if x else '-', '%x' % y['tile'] if y else '-',
            '%.0f' % (y['flops'] / (y['ms'] * 1e-3) / 1e12) if y else '-'))
    print('total %.1f %.1f us' % (ta, tb))


if __name__ == '__main__':
    main()
