"""MI355X-native SelectiveUNet_B training path (drop-in for the reference's
`model.UNet_B`, `selective_loss.calc_selective_risk_image_b` and `train.py`)."""
