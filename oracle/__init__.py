"""CPU oracle for the quantized LLaMA decode path — TEST INFRASTRUCTURE ONLY.

A numpy restatement of the reference algorithm (if001/lit-llama-ja @ 2025-02-05), each
function citing the reference file:line it follows. It is the checker for the HIP path
and the `cpu_baseline` ("port") leg of bench.py. Only tests/, bench.py's cpu_baseline leg
and __graft_entry__.smoke() may import it; the product package (lit-llama-ja_amd/) never
does, and fails loudly instead of falling back to it.

Pinning: fp32 model/ops, ColBlockQuantizedLinear int4/int8 and the generate() loop are
pinned against fixtures produced by the reference itself (tests/golden/make_golden.py,
tests/test_oracle_golden.py). LLM.int8() (bitsandbytes, absent from the image and
un-vendored in the reference, requirements.txt:7 unpinned) is restated from its published
algorithm: that part is "parity unpinned".
"""
