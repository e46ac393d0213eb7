"""lodestar_amd: MI355X-native BLS12-381 signature-set batch verifier for
Lodestar's IBlsVerifier hot path."""
__all__ = ["native", "verifier"]
