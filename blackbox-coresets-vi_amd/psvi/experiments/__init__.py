"""Data and results plumbing of the reference's psvi/experiments (SURVEY §8(f)
rank 4): offline datasets, the results dict and its files, and a
flow_psvi-style driver over the methods the HIP path runs."""
from .experiments_utils import (SynthDataset, make_four_class_dataset, make_mnist_shaped,  # noqa: F401
                                make_synthetic, make_synthetic_normal, read_dataset, rec_dd,
                                split_data, write_to_files)
from .flow_psvi import experiment_driver, inf_dict  # noqa: F401
