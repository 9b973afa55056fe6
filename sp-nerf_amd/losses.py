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
    """Subset depth loss (usealldepth=False — the trainer's default, opt.py:79 — MSE form,
    metrics.py:82-132,151-153).

    The reference selects the valid rays, then the rays outside the expected distribution,
    and returns λ/3 · mean((n_apply / B) · tw · (pd − td)²) over the selected rays, i.e.
    λ/3 · Σ_{valid ∧ apply} tw · (pd − td)² / B (0 when nothing is selected).  The same sum is
    taken here with a 0/1 mask instead of boolean indexing, so it needs no host sync (boolean
    indexing is a device→host count) and can be captured in a HIP graph.  The predicted std
    only enters the comparison, so no gradient flows through its sqrt."""

    def __init__(self, lambda_ds=1.0):
        super().__init__()
        self.lambda_ds = lambda_ds / 3.0

    def forward(self, inputs, target_depth, target_weight, target_valid_depth, target_std):
        z = inputs["z_vals_coarse"]
        pd = inputs["depth_coarse"]
        pw = inputs["weights_coarse"]
        with torch.no_grad():
            pstd = (((z - pd.unsqueeze(-1)).pow(2) * pw).sum(-1)).sqrt()
            apply = (target_valid_depth > 0) & torch.logical_or((pd - target_depth).abs() > target_std,
                                                                pstd > target_std)
            m = apply.to(pd.dtype)
        loss = self.lambda_ds * torch.sum(m * target_weight * (pd - target_depth) ** 2) / float(pd.shape[0])
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
