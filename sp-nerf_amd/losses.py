"""Training losses over the render dictionary — mirrors modules/metrics.py of the reference
(SNerfLoss :27-45, solar_correction :17-24, DepthLoss :68-159, SemanticLoss :162-183, psnr
:206-207).  Plain torch ops on (B, ·) tensors; the per-point work stays in the HIP kernels.
(A fused loss + composite-backward kernel is the next §8(f) row.)"""
from __future__ import annotations

import torch


def solar_correction(loss_dict, inputs, typ, lambda_sc=0.05):
    sun_sc = inputs[f"sun_sc_{typ}"].squeeze()
    term2 = torch.sum(torch.square(inputs[f"transparency_sc_{typ}"].detach() - sun_sc), -1)
    term3 = 1 - torch.sum(inputs[f"weights_sc_{typ}"].detach() * sun_sc, -1)
    loss_dict[f"{typ}_sc_term2"] = lambda_sc / 3.0 * torch.mean(term2)
    loss_dict[f"{typ}_sc_term3"] = lambda_sc / 3.0 * torch.mean(term3)
    return loss_dict


class SNerfLoss(torch.nn.Module):
    def __init__(self, lambda_sc=0.05):
        super().__init__()
        self.lambda_sc = lambda_sc
        self.loss = torch.nn.MSELoss(reduction="mean")

    def forward(self, inputs, targets):
        loss_dict = {"coarse_color": self.loss(inputs["rgb_coarse"], targets)}
        if self.lambda_sc > 0:
            loss_dict = solar_correction(loss_dict, inputs, "coarse", self.lambda_sc)
        return sum(loss_dict.values()), loss_dict


class DepthLoss(torch.nn.Module):
    """Subset depth loss (usealldepth=False, MSE form, metrics.py:82-132,151-153)."""

    def __init__(self, lambda_ds=1.0):
        super().__init__()
        self.lambda_ds = lambda_ds / 3.0

    def forward(self, inputs, target_depth, target_weight, target_valid_depth, target_std):
        valid = target_valid_depth > 0
        z = inputs["z_vals_coarse"][valid]
        pd = inputs["depth_coarse"][valid]
        pw = inputs["weights_coarse"][valid]
        pstd = (((z - pd.unsqueeze(-1)).pow(2) * pw).sum(-1)).sqrt()
        tw, td, ts = target_weight[valid], target_depth[valid], target_std[valid]
        apply = torch.logical_or((pd - td).abs() > ts, pstd > ts)
        n_apply = apply.sum()
        scale = n_apply.float() / float(target_valid_depth.shape[0])
        per = tw[apply] * (pd[apply] - td[apply]) ** 2
        loss = self.lambda_ds * torch.mean(scale * per) if per.numel() else pd.sum() * 0.0
        return loss, {"coarse_ds": loss}


class SemanticLoss(torch.nn.Module):
    def __init__(self, lambda_ss=1.0):
        super().__init__()
        self.lambda_ss = lambda_ss
        self.ce = torch.nn.CrossEntropyLoss(ignore_index=-100)

    def forward(self, inputs, targets):
        loss = self.lambda_ss * self.ce(inputs["sem_logits_coarse"], targets)
        return loss, {"coarse_ss": loss}


def psnr(image_pred, image_gt):
    return -10 * torch.log10(torch.mean((image_pred - image_gt) ** 2))
