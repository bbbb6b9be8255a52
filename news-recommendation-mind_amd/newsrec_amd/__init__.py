"""newsrec_amd — MI355X-native two-tower news-recommendation train/score path.

Host-side mirror of tyh666/News-Recommendation-MIND's model interface (models/Embeddings,
models/Encoders, models/Modules/Attention.py, models/TwoTowerBaseModel.py) whose compute
runs in libnewsrec_hip.so (hand-written HIP for gfx950) through a C ABI.
"""
__version__ = "0.1.0"
