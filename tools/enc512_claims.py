"""Correlate k_enc512 claims (CHECK build printf 'CLAIM n x seg xcc') with bad images."""
import re
import sys
claims, bad = {}, []
for line in open(sys.argv[1]):
    m = re.match(r"CLAIM (\d+) (\d+) (-?\d+) (\d+)", line)
    if m:
        claims[int(m.group(1))] = (int(m.group(2)), int(m.group(3)), int(m.group(4)))
    m = re.search(r"first rows (\[[^\]]*\])", line)
    if m and not bad:
        bad = eval(m.group(1))
print("claims", len(claims))
from collections import Counter
print("per xcd", sorted(Counter(v[0] for v in claims.values()).items()))
print("bad rows (image, xcd, seg):", [(b, *claims.get(b, (None, None, None))[:2]) for b in bad])
