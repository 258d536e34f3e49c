"""Built-in preprocessors. Parity: reference python/ray/data/preprocessors/*."""
from ray_memory_management_amd.data.preprocessors.basic import (  # noqa: F401
    BatchMapper, Categorizer, Chain, Concatenator, CountVectorizer, FeatureHasher, HashingVectorizer,
    LabelEncoder, MaxAbsScaler, MinMaxScaler, MultiHotEncoder, Normalizer, OneHotEncoder, OrdinalEncoder,
    PowerTransformer, RobustScaler, SimpleImputer, StandardScaler, Tokenizer)

__all__ = ["BatchMapper", "Categorizer", "Chain", "Concatenator", "CountVectorizer", "FeatureHasher",
           "HashingVectorizer", "LabelEncoder", "MaxAbsScaler", "MinMaxScaler", "MultiHotEncoder", "Normalizer",
           "OneHotEncoder", "OrdinalEncoder", "PowerTransformer", "RobustScaler", "SimpleImputer", "StandardScaler",
           "Tokenizer"]
