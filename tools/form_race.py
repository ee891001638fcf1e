"""Diagnosis: the f32 s-seg forward at B = 3 under VA_CONV3T forms 2 / 6, laned and serial, repeated -- which
combination ever differs from the serial form-2 forward (a timing-dependent race shows up as a run that differs).
python tools/form_race.py ITERS [FORMS, e.g. 2,0,5]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from vision_assist_amd.seg import SegNet
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    arch = Arch("s")
    net = SegNet(arch, fold(arch, synthetic_state_dict(arch, seed=5)), dtype="f32")
    frames = torch.randint(0, 256, (3, 640, 640, 3), generator=torch.Generator().manual_seed(11),
                           dtype=torch.uint8).cuda()
    plans = {lanes: net.plan(3, 640, 640, tag=int(lanes), lanes=lanes) for lanes in (False, True)}

    def run(form, lanes):
        os.environ["VA_CONV3T"] = form
        p = plans[lanes]
        p["frames"].copy_(frames)
        net.run_plan(p)
        torch.cuda.synchronize()
        return [t.clone() for t in p["out"].levels] + [p["out"].proto.clone()]

    ref = run("2", False)
    bad = {}
    for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
        for form in (sys.argv[2].split(",") if len(sys.argv) > 2 else ("2", "6", "5")):
            for lanes in (False, True):
                got = run(form, lanes)
                d = [float((g - r).abs().max()) for g, r in zip(got, ref)]
                if any(v != 0 for v in d):
                    bad.setdefault(f"form{form}_lanes{int(lanes)}", []).append((it, d))
    print(json.dumps({"mismatches": bad}, indent=1))


if __name__ == "__main__":
    main()
