"""spnerf_amd — MI355X (gfx950) volumetric render path for SP-NeRF.

Drop-in for the reference's render surface:

* ``render_rays``, ``sample_pdf``, ``sample_3sigma``, ``compute_samples_around_depth``,
  ``GenerateGuidedSamples``  (modules/rendering.py)
* ``SPNeRF``, ``inference``, ``Mapping``, ``Siren``, ``sine_init``, ``first_layer_sine_init``
  (models/spnerf.py) and ``load_model`` (models/__init__.py)

all backed by the hand-written HIP kernels of ``libspnerf_amd.so`` (C ABI:
include/spnerf_amd.h).  Importing the package does not touch the GPU; the first compute
call loads the library and raises if it is missing or if tensors are on the CPU.
"""
from .rendering import (GenerateGuidedSamples, compute_samples_around_depth, render_rays, sample_3sigma,  # noqa: F401
                        sample_pdf, stratified)
from . import optim  # noqa: F401  (optim.Adam: the library's one-launch Adam step)
from . import dsm  # noqa: F401  (DSM extraction: satellite_scene.py:475-568 on the GPU)
from .rng import PhiloxRandom, ReplayRandom, TorchRandom, current_random_source, random_source, set_random_source  # noqa: F401
from .spnerf import (SPNeRF, Mapping, Siren, first_layer_sine_init, inference, inference_rays, run_mlp,  # noqa: F401
                     sine_init)

__version__ = "0.1.0"


def load_model(args):
    """models/__init__.py:4-16."""
    if args.model == "sp-nerf":
        return SPNeRF(num_sem_classes=args.num_sem_classes, s_embedding_factor=args.s_embedding_factor,
                      layers=args.fc_layers, feat=args.fc_units, mapping=args.mapping,
                      t_embedding_dims=args.t_embbeding_tau, beta=args.beta, sem=args.sem,
                      precision=getattr(args, "mlp_precision", "fp32"))
    raise ValueError(f'model {args.model} is not valid')
