from .synthetic import Dataset, IdxMNIST, SyntheticMNIST, SyntheticTokens, batch_ranges

__all__ = ["Dataset", "IdxMNIST", "SyntheticMNIST", "SyntheticTokens", "batch_ranges"]
