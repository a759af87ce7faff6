"""MI355X-native exact k-NN search path for AAPPHH/image_recommender.

Drop-in for the reference's faiss hot path: ``faiss_compat`` (the faiss object
protocol over the C ABI of ``include/imgrec_knn.h``), the reference's build/search modules under
``main/``, the colour-histogram extractor under ``vector_scripts/``, and ``sharded`` (row-sharded
multi-GPU index merged through an RCCL all-gather).
"""
__version__ = "0.1.0"
