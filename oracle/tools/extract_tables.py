"""Dev-time provenance tool (never run on the GPU box, never imported by the product).

Reads the piece tables of the reference (`src/map.cpp:446-695`) and re-encodes them as
one-byte hex codes for `gym-eldorado_amd/csrc/cog_tables.h`:
    code = (requirement << 3) | n        (requirement: M=0,P=1,C=2,DISCARD=3,REMOVE=4,NULL=5)
    bit 6 = is_end
For NULL hexes the low 3 bits hold `player_start` (unobservable for NULL hexes).
Usage: python oracle/tools/extract_tables.py /root/reference/src/map.cpp
"""
import re, sys

src = re.sub(r"//[^\n]*", "", open(sys.argv[1]).read())
KIND = {"jungle": 0, "water": 1, "desert": 2, "rubble": 3, "basecamp": 4}

def code(tok):
    tok = tok.strip()
    if tok == "&mountain":
        return 40
    m = re.fullmatch(r"&start_hexes\[(\d)\]", tok)
    if m:
        return 40 | (int(m.group(1)) + 1)
    m = re.fullmatch(r"&end_hexes\[(\d)\]", tok)
    if m:  # end_hexes = {PADDLE 1 end, MACHETE 1 end}  (map.cpp:121-122)
        return [(1 << 3) | 1 | 64, (0 << 3) | 1 | 64][int(m.group(1))]
    m = re.fullmatch(r"&(\w+)\[(\d)\]", tok)
    return (KIND[m.group(1)] << 3) | (int(m.group(2)) + 1)

blocks = re.findall(r"MapPiece\(\s*\{(.*?)\}\s*,\s*(\w+)\s*,\s*Difficulty::(\w+)\s*,\s*PieceType::(\w+)\s*,\s*PieceSize::(\w+)\)", src, re.S)
out = []
for hexes, coords, diff, ptype, size in blocks:
    toks = [t for t in hexes.replace("\n", " ").split(",") if t.strip()]
    out.append((list(map(code, toks)), coords, diff, ptype, size))
for h, c, d, t, s in out:
    print(len(h), c, d, t, s, ",".join(str(x) for x in h))
