"""Static instruction-class counts of device kernels in a hipcc -S listing
(--cuda-device-only), optionally split at `; sec:` markers placed with
asm volatile("; sec: name") in the source.
    python tools/isa_count.py listing.s <kernel-substring> [...]"""
import collections
import sys


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("s_waitcnt", "s_barrier", "s_cbranch", "s_branch", "s_nop", "s_endpgm", "s_setprio", "s_sleep")):
        return "misc"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem_st" if "store" in op else "vmem_ld"
    return "other"


def kernel_body(text, sub):
    lines = text.split("\n")
    for i, ln in enumerate(lines):
        if ln.startswith("_Z") and ln.split(":")[0].find(sub) >= 0 and ln.rstrip().endswith(ln.split(":")[0] + ":" + ln.split(":", 1)[1]) :
            start = i
            break
    else:
        raise SystemExit(f"kernel {sub} not found")
    out = []
    for ln in lines[start + 1:]:
        if ln.startswith(".Lfunc_end"):
            break
        out.append(ln)
    return out


def main():
    text = open(sys.argv[1]).read()
    for sub in sys.argv[2:]:
        sec = "all"
        counts = collections.OrderedDict()
        for ln in kernel_body(text, sub):
            t = ln.strip()
            if t.startswith("; sec:"):
                sec = t.split(":", 1)[1].strip()
                continue
            if not t or t.startswith((";", ".")) or t.endswith(":"):
                continue
            counts.setdefault(sec, collections.Counter())[classify(t.split()[0])] += 1
        print(sub)
        tot = collections.Counter()
        for k, c in counts.items():
            tot.update(c)
            print(f"  {k:24s} {dict(sorted(c.items()))}  = {sum(c.values())}")
        print(f"  {'TOTAL':24s} {dict(sorted(tot.items()))}  = {sum(tot.values())}")


if __name__ == "__main__":
    main()
