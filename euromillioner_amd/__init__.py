"""euromillioner_amd — MI355X-native lottery-draw prediction trainer.

A from-scratch, AMD Instinct MI355X (gfx950 / CDNA4) framework with the
capabilities of mareksagan/Euromillioner: draw ingestion (CSV / synthetic /
offline HTML table), a positional 70/30 split, XGBoost-semantics gradient-boosted
trees, a random forest, and 62-in/62-out MLPs trained with hand-written HIP
kernels, RCCL data parallelism and DL4J-ModelSerializer checkpoints.
"""
__version__ = "0.1.0"
