"""Instruction mix of kernels in a hipcc --cuda-device-only -S listing: python scripts/asm_mix.py FILE.s name..."""
import re
import sys

txt = open(sys.argv[1]).read()
PAT = (r"v_mfma\w+|v_exp_f32|v_permlane\w+|ds_read\w+|ds_write\w+|v_cvt_pk_bf16_f32|v_maximum3_f32|s_barrier|"
       r"buffer_load\w+|buffer_store\w+|global_store\w+|global_load\w+|s_waitcnt|v_pk_\w+|v_mul_f32|v_fma_f32|v_add_f32|"
       r"s_nop|v_accvgpr\w+|scratch_\w+|s_cbranch\w+")
for fn in sys.argv[2:]:
    m = re.search(r"\n(_Z\w*" + fn + r"\w*):[^\n]*\n(.*?)\.Lfunc_end", txt, re.S)
    if not m:
        print(fn, "not found")
        continue
    cnt = {}
    lines = [l for l in m.group(2).split("\n") if l.strip() and not l.strip().startswith((";", "."))]
    for l in lines:
        mm = re.match(r"\s*(" + PAT + r")\b", l)
        if mm:
            k = mm.group(1)
            cnt[k] = cnt.get(k, 0) + 1
    print(m.group(1), "instructions", len(lines))
    print("   ", dict(sorted(cnt.items())))
