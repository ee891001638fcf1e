"""CPU check of the algebra behind va_conv_args.mode 2: proto's ConvTranspose2d(k2, s2) -> 3x3 conv
equals four sub-pixel 2x2 convs over the low-res map with the folded weights (float64, exact to
rounding), including the border pixels where the deconv bias must only count taps inside the map."""
import torch
import torch.nn.functional as F


def test_subpixel_fold_equals_deconv_then_conv3x3():
    from vision_assist_amd.seg import fold_proto_weights
    g = torch.Generator().manual_seed(7)
    ci, c, o, H, W = 16, 12, 8, 5, 7
    wd = torch.randn(ci, c, 2, 2, generator=g, dtype=torch.float64)
    bd = torch.randn(c, generator=g, dtype=torch.float64)
    w2 = torch.randn(o, c, 3, 3, generator=g, dtype=torch.float64)
    x = torch.randn(2, ci, H, W, generator=g, dtype=torch.float64)
    ref = F.conv2d(F.conv_transpose2d(x, wd, bd, stride=2), w2, None, padding=1)  # [2, o, 2H, 2W]
    wc = fold_proto_weights(wd, bd, w2)                                            # [4, o, 2, 2, ci + 8]
    assert wc.shape == (4, o, 2, 2, ci + 8)
    xe = torch.cat([x, torch.ones(2, 1, H, W, dtype=torch.float64), torch.zeros(2, 7, H, W, dtype=torch.float64)], 1)
    xp = F.pad(xe, (1, 1, 1, 1))  # zero padding: the ones channel is 0 outside the map
    for dy in range(2):
        for dx in range(2):
            k = wc[2 * dy + dx].permute(0, 3, 1, 2)  # [o, ci + 8, 2, 2]
            got = F.conv2d(xp[:, :, dy:dy + H + 1, dx:dx + W + 1], k)
            assert got.shape == (2, o, H, W)
            assert torch.allclose(got, ref[:, :, dy::2, dx::2], atol=1e-10, rtol=1e-10)
