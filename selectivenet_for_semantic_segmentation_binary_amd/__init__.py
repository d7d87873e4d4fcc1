"""MI355X-native SelectiveUNet_B training path.

Drop-in replacements for the reference's hot path (yellofi/SelectiveNet_for_semantic_segmentation_binary):

* `UNet_B`, `CBR_2D`                    <- model.py:9-103
* `UNet` (CE variant)                   <- model.py:105-191
* `calc_selective_risk_image_b`         <- selective_loss.py:58-85
* `calc_selective_risk_image`           <- selective_loss.py:24-56
* `BCEWithLogitsLoss`                   <- torch.nn.BCEWithLogitsLoss (train.py:78)
* `CrossEntropyLoss`                    <- torch.nn.CrossEntropyLoss (train.py:80)
* `Adam`                                <- torch.optim.Adam (train.py:90)
* `parallel.init_data_parallel`         <- torch.nn.DataParallel (train.py:131-134)

All compute runs in libselunet.so (HIP, gfx950); there is no CPU fallback.
"""
from .layout import count_params, state_dict_keys  # noqa: F401
from .model import CBR_2D, UNet, UNet_B  # noqa: F401
from .optim import Adam  # noqa: F401
from .selective_loss import (BCEWithLogitsLoss, CrossEntropyLoss, calc_selective_risk_image,  # noqa: F401
                             calc_selective_risk_image_b)
from . import parallel  # noqa: F401

__version__ = "0.1.0"
