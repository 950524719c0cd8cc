"""butterfly_amd — MI355X-native distributed transformer inference (Butterfly capabilities)."""
__version__ = "0.1.0"
