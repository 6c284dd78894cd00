"""tossctr -- MI355X-native DARE + QNN-alpha CTR training hot path (drop-in for the reference's
src/models/wrapper.py CTRModel and the src/train.py step), compute in libctrhip.so (gfx950 HIP)."""
from .arch import Arch
from .optim import ArenaEMA, FusedAdamW, build_ema
from .wrapper import CTRModel

__all__ = ["Arch", "CTRModel", "FusedAdamW", "ArenaEMA", "build_ema"]
