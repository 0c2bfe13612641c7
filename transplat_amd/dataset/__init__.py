"""Host-side test-data plumbing: the `.torch` chunk reader and its crop shim."""
from .re10k_chunks import EXPERIMENTS, ChunkDatasetCfg, ChunkTestDataset, convert_poses  # noqa: F401
