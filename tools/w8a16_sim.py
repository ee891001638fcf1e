"""Would a W8A16 form of C5 (e4m3 weights, one scale per output channel as seg.py _pack_fp8 packs them, activations
kept at higher precision) reach VERDICT r4's chain bar?  CPU simulation, no kernel: the fp32 oracle chain
(tests/chain_util.oracle_sequence) run with every conv's weights quantized to e4m3 and back (model.0 excepted: the
fp8 plan keeps it bf16), activations in fp32 -- an optimistic bound for a bf16-activation kernel -- compared with
the fp32 oracle chain fixture c5/<regime> (tests/golden/chain_oracle.json.gz) by tests/chain_util.compare / rates.
Also the forward's relative L2 per head against fp32.   python tools/w8a16_sim.py [dense_box|sparse] [frames]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def quantize_e4m3(fw: dict) -> dict:
    out = {}
    for k, v in fw.items():
        if not (isinstance(v, tuple) and len(v) == 2 and v[0].dim() == 4) or k == "model.0":
            out[k] = v
            continue
        w, b = v
        wf = w.float()
        amax = wf.abs().flatten(1).amax(1)
        s = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax)).view(-1, 1, 1, 1)
        q = (wf / s).clamp(-448, 448).to(torch.float8_e4m3fn).float() * s
        out[k] = (q.to(w.dtype), b)
    return out


def main():
    from oracle import yolo_ref as Y
    from tests.chain_util import compare, frame_batch, load_fixture, oracle_sequence, rates, weights
    regime = sys.argv[1] if len(sys.argv) > 1 else "dense_box"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    torch.set_num_threads(8)
    arch, fw = weights(regime, scale="m")
    fq = quantize_e4m3(fw)
    frames = frame_batch(8000, 8, 1280)[:n]
    with torch.no_grad():
        ref = Y.forward(arch, fw, Y.preprocess(frames[:2]))
        got = Y.forward(arch, fq, Y.preprocess(frames[:2]))
    l2 = {k: round(((g - r).norm() / r.norm()).item(), 4) for k, g, r in zip(("box", "cls", "coef", "proto"), got, ref)}
    want = load_fixture(f"c5/{regime}")[:n]
    recs = oracle_sequence(arch, fq, frames)
    cmps = [compare(g, w, f32=False) for g, w in zip(recs, want)]
    print(json.dumps({"form": "W8A16 simulation (e4m3 weights per output channel, fp32 activations)",
                      "regime": regime, "frames": n, "forward_rel_l2_vs_fp32": l2, "chain": rates(cmps)}), flush=True)


if __name__ == "__main__":
    main()
