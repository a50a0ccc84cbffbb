"""pinot_amd: MI355X-native execution path for Pinot's pinot-core segment query hot path.

Host-side mirror of the reference's PlanMaker / Operator / AggregationFunction interface over the
libpgx C-ABI (include/pgx.h).  See DESIGN.md.
"""
__version__ = "0.1.0"
