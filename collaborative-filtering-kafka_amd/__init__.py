"""MI355X-native ALS engine for the Collaborative-Filtering-Kafka hot path.

The directory name contains dashes, so it is loaded under the module name ``cfk_amd`` (see
``load_package`` in ``__graft_entry__.py``). The native library is ``build/libcfk_als.so``.
"""
from .engine import ALSEngine, Dataset, factor_stride, u01, write_prediction_csv, write_prediction_matrix_csv  # noqa: F401
from .engine import decode_feature_message, decode_id_rating, encode_feature_message, encode_id_rating  # noqa: F401
from ._lib import ALSError  # noqa: F401
from .app import ALSApp  # noqa: F401
