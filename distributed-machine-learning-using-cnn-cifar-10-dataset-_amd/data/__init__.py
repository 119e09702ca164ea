"""Input pipeline: CIFAR-10 binary records (native reader) and synthetic data."""
from .cifar import (batches_dir, dataset, load_cifar10, prepare, read_records, resolve_data_dir,  # noqa: F401
                    synthetic, write_records)
