"""CPU check of tools/shift64_top_vgpr.hip's assembly: every k_parse<TOP, PIN>
kernel allocates the VGPRs and reads its left shifts' amount from the register
its experiment needs (prints one line per kernel; exit 1 on a mismatch).

    python3 tools/shift64_asm_check.py shift64_top_vgpr.s
"""
import re
import sys

# (TOP, PIN) -> (allocation, amount register of the two v_lshlrev_b64); None: any
WANT = {("0", "n1"): (24, None), ("0", "4"): (24, "v4"), ("0", "23"): (24, "v23"),
        ("32", "23"): (32, "v23"), ("32", "31"): (32, "v31"), ("40", "31"): (40, "v31")}


def main(path):
    ok = True
    seen = set()
    for blk in re.split(r"\n(?=_Z\S*:)", open(path).read()):
        m = re.match(r"_Z7k_parseILi(\d+)ELi(n?\d+)E\S*:", blk)
        if not m:
            continue
        key = m.groups()
        seen.add(key)
        n = int(re.search(r"; NumVgprs: (\d+)", blk).group(1))
        alloc = (n + 7) // 8 * 8
        amts = re.findall(r"\tv_lshlrev_b64\s+\S+, (\S+), ", blk)
        want_alloc, want_amt = WANT[key]
        good = alloc == want_alloc and len(amts) == 2 and (want_amt is None or set(amts) == {want_amt})
        top = f"v{alloc - 1}"
        print(f"k_parse<{key[0]}, {key[1].replace('n', '-')}>: vgprs {n} alloc {alloc} left-shift amounts {amts} "
              f"(top of allocation {top}: {'yes' if top in amts else 'no'}) {'ok' if good else 'MISMATCH'}")
        ok &= good
    ok &= seen == set(WANT)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
