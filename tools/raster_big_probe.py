"""Large-image rasterizer parity probe: kernel vs literal oracle for a few (Gaussians, resolution,
sort) settings; prints L-inf over unflagged pixels, the worst pixel and its tile's list length."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from oracle import raster as oracle_raster  # noqa: E402
from transplat_amd import synthetic as S  # noqa: E402
from transplat_amd.model.decoder.hip_splatting import prepare_cameras, rasterize  # noqa: E402

dev = torch.device("cuda:0")
CASES = [(128, (1024, 1024)), (128, (1280, 1280)), (64, (1280, 1280)), (128, (512, 512)), (128, (768, 768))]
if len(sys.argv) > 1:  # ctx:h:w ...
    CASES = [(int(a), (int(b), int(c))) for a, b, c in (x.split(":") for x in sys.argv[1:])]
for ctx, hw in CASES:
    g = S.make_gaussians(1, image_shape=(ctx, ctx))
    b = S.make_batch(1, num_target=1, image_shape=hw)
    t = b["target"]
    cams = prepare_cameras(t["extrinsics"].reshape(1, 4, 4), t["intrinsics"].reshape(1, 3, 3), t["near"].reshape(-1),
                           t["far"].reshape(-1), torch.zeros(1, 3))
    ref, rr, counts, pflag, gflag = oracle_raster.render_flagged(g["means"], g["covariances"], g["harmonics"],
                                                                 g["opacities"], cams, hw, 1, 3)
    gd = {k: v.to(dev) for k, v in g.items()}
    col, rad = rasterize(gd["means"], gd["covariances"], gd["harmonics"], gd["opacities"], cams.to(dev), hw, 1,
                         sh_degree=3)
    col = col.cpu().numpy()
    err = np.abs(col - ref).max(axis=1)[0]
    clear = pflag[0] == 0
    e2 = np.where(clear, err, 0)
    y, x = np.unravel_index(np.argmax(e2), e2.shape)
    nbad = int((e2 > 1e-4).sum())
    print(f"ctx {ctx} G={g['means'].shape[1]} hw={hw}: L-inf {e2.max():.3e} at ({y},{x}) tile ({y // 16},{x // 16}); "
          f"{nbad} unflagged px > 1e-4; flagged {int((pflag != 0).sum())}; ambiguous radii {int(gflag.sum())}; "
          f"rendered {counts}; radii diff {(rad.cpu().numpy() != rr).sum()}", flush=True)
    if nbad:
        ys, xs = np.nonzero(e2 > 1e-4)
        tiles = sorted(set(zip((ys // 16).tolist(), (xs // 16).tolist())))
        print("   bad tiles:", tiles[:20], "n", len(tiles))
