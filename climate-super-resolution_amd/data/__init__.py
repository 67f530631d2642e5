"""On-device data pipeline: the per-sample work of the reference's
``ClimateDataset`` done for a whole batch of raw tiles in HBM by ``libclimsr_hip.so``."""
from .tile_pipeline import DeviceTilePipeline, TransformsCfg  # noqa: F401
