"""tools/kernel_resources.py reads the compiler's kernel-resource remarks (CPU, synthetic remarks)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import kernel_resources  # noqa: E402

TAG = " [-Rpass-analysis=kernel-resource-usage]"


def _remarks(sym, vgprs, lds):
    lines = [f"x.hip:1:1: remark: Function Name: {sym}{TAG}"]
    for k, v in (("TotalSGPRs", 106), ("VGPRs", vgprs), ("AGPRs", 0), ("ScratchSize [bytes/lane]", 0),
                 ("Dynamic Stack", "False"), ("Occupancy [waves/SIMD]", 2), ("SGPRs Spill", 5),
                 ("VGPRs Spill", 0), ("LDS Size [bytes/block]", lds)):
        lines.append(f"x.hip:1:1: remark:     {k}: {v}{TAG}")
    return "\n".join(lines)


def test_parse_names_the_element_instantiation():
    text = "\n".join([_remarks("_ZN2hk14k_element_pipeILb1ELb0ELb1ELb1ELi3ELb1ELi2EEEvNS_8ElemArgsE", 256, 59008),
                      "noise line",
                      _remarks("_ZN2hk4k_bcENS_6BCArgsE", 40, 0)])
    ks = kernel_resources.parse(text)
    assert len(ks) == 2
    e = ks[0]
    assert e["kernel"] == "k_element_pipe" and e["mode"] == "reference_order" and e["assembly"] == "owner OS=2"
    assert e["args"]["NT"] == 3 and e["args"]["DO_DELETE"] is True and e["args"]["STORE_TRIAX"] is False
    assert e["vgprs"] == 256 and e["lds_static_bytes"] == 59008 and e["waves_per_simd"] == 2
    assert e["dynamic_stack"] is False and e["sgpr_spill"] == 5
    assert ks[1]["kernel"] == "k_bc" and ks[1]["vgprs"] == 40
