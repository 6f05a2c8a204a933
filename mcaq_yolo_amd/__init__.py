"""MI355X-native MCAQ spatial-adaptive-quantization hook path (gfx950 HIP)."""
