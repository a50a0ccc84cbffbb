"""Server response and broker reduce for the segment query path: the step after the combine.

A server answers an instance request with ONE response per query (the reference's DataTable, built by
InstanceResponseOperator from the combined IntermediateResultsBlock, core/operator/InstanceResponseOperator.java); the
broker merges the responses of all servers and renders the final answer (BrokerReduceService.reduceOnDataTable,
core/query/reduce/BrokerReduceService.java:62-256).  Here:

* ``ServerQueryExecutor.process_query`` runs the inter-segment plan of ``engine.InstancePlanMakerImplV2`` (the GPU
  path) and wraps the combined block in an ``InstanceResponse``: the aggregation intermediates (count as int, sum / min /
  max as double, avg as (sum, count)) or, for group-by, the trimmed combine maps (one {group string: intermediate} per
  function), plus the four execution statistics and any processing exception (ServerQueryExecutorV1Impl.java:118-176).
  ``datatable.response_to_datatable`` serializes it as the reference's DataTable bytes (version 2, custom ser/de;
  common/utils/DataTable.java:315-482) and the reduce accepts either form.
* ``BrokerReduceService.reduce_on_data_table`` sums the statistics, turns exception responses into processing
  exceptions, reduces aggregation results with each function's ``reduce`` and group-by maps with ``combineTwoValues``
  + ``reduce`` (query/aggregation/groupby/AggregationGroupByOperatorService.java:93-129), keeps the top N groups per
  function (MIN ascending, others descending: GroupByResultComparator, :405-440) and formats double values with
  ``%1.5f`` and long values with ``toString`` (BrokerReduceService.formatValue, :293-296).
"""
from __future__ import annotations

import decimal
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from . import engine as E
from . import extended as X
from .pql import EXT_FUNCTIONS


_NAMES = {"distinctcount": "distinctCount", "distinctcounthll": "distinctCountHLL", "fasthll": "fasthll", "minmaxrange": "minMaxRange"}


def function_name(agg: dict) -> str:
    """AggregationFunction.getFunctionName: count_star, sum_<col>, min_<col>, max_<col>, avg_<col>, distinctCount_<col>,
    minMaxRange_<col>, percentileNN_<col> (query/aggregation/function/CountAggregationFunction.java:118-120,
    SumAggregationFunction.java:207-209, DistinctCountAggregationFunction.java:165, MinMaxRangeAggregationFunction
    .java:170, quantile/PercentileAggregationFunction.java:171)."""
    fn = base_function(agg["fn"])
    if fn == "count":  # COUNTMV too: registered as CountAggregationFunction (AggregationFunctionRegistry.java:76)
        return "count_star"
    if fn.startswith("percentileest"):  # DigestAggregationFunction.getFunctionName (:161-163)
        return "percentileEst%s_%s" % (fn[len("percentileest"):], agg["column"])
    return "%s_%s" % (_NAMES.get(fn, fn), agg["column"])


def java_format_5f(x: float) -> str:
    """String.format(Locale.US, "%1.5f", double): Java rounds the shortest decimal representation of the double
    (Double.toString digits) HALF_UP, where C's printf rounds the exact binary value; infinities print as
    (-)Infinity and NaN as NaN."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    d = decimal.Decimal(repr(float(x))).quantize(decimal.Decimal("0.00001"), rounding=decimal.ROUND_HALF_UP)
    s = format(d, "f")
    return "-0.00000" if s == "0.00000" and math.copysign(1.0, x) < 0 else s


# {Count,Sum,Min,Max,Avg}MVAggregationFunction combine / reduce like their single-value counterparts (the values of
# every doc fold into the same intermediates: count, double sum, min, max, AvgPair)
_MV_BASE = {"countmv": "count", "summv": "sum", "minmv": "min", "maxmv": "max", "avgmv": "avg"}


def base_function(fn: str) -> str:
    """The legacy function class a request key maps to: AggregationFunctionRegistry.java:76-91 registers every *mv key
    with its single-value class (names, combine and reduce are the base function's)."""
    return _MV_BASE.get(fn) or X.base_fn(fn)


def _combine_two(fn: str, a, b):
    """combineTwoValues of the legacy functions (CountAggregationFunction.java:79-87 long add, SumAggregationFunction
    .java:168-176 double add, MinAggregationFunction.java:112-120, Max..., AvgAggregationFunction.java:116-125 pair add);
    a null side yields the other."""
    if a is None:
        return b
    if b is None:
        return a
    fn = base_function(fn)
    if fn in EXT_FUNCTIONS:
        return X.combine_two(fn, a, b)
    if fn == "count":
        return int(a) + int(b)
    if fn == "sum":
        return float(a) + float(b)
    if fn == "min":
        return a if a < b else b
    if fn == "max":
        return a if a > b else b
    return (float(a[0]) + float(b[0]), int(a[1]) + int(b[1]))


def _reduce(fn: str, values: Sequence):
    """AggregationFunction.reduce: count -> long sum; sum -> double sum; min / max over the default +/-inf; avg -> sum /
    count, 0.0 when no docs (AvgAggregationFunction.java:128-143)."""
    fn = base_function(fn)
    if fn in EXT_FUNCTIONS:  # combine the intermediates, then the function's final value
        acc = None
        for v in values:
            acc = v if acc is None else X.combine_two(fn, acc, v)
        if acc is None:
            return 0 if fn in ("distinctcount", "distinctcounthll", "fasthll") else (-1.0 if fn == "minmaxrange" else 0.0)
        return X.reduce_value(fn, acc)
    if fn == "count":
        return sum(int(v) for v in values)
    if fn == "sum":
        s = 0.0
        for v in values:
            s += float(v)
        return s
    if fn == "min":
        m = math.inf
        for v in values:
            if v < m:
                m = float(v)
        return m
    if fn == "max":
        m = -math.inf
        for v in values:
            if v > m:
                m = float(v)
        return m
    s, c = 0.0, 0
    for v in values:
        s += float(v[0])
        c += int(v[1])
    return s / c if c > 0 else 0.0


def _format(fn: str, v) -> str:
    """Long / Integer (count, distinctcount) -> toString; doubles -> %1.5f (BrokerReduceService.formatValue)."""
    fn = base_function(fn)
    return str(int(v)) if fn in ("count", "countmv", "distinctcount", "distinctcounthll", "fasthll") \
        or fn.startswith("percentileest") \
        else java_format_5f(float(v))


@dataclass
class InstanceResponse:
    """One server's answer (the DataTable's content): aggregation intermediates, or trimmed group-by maps."""
    aggregation: Optional[list] = None
    group_by: Optional[List[Dict[str, object]]] = None
    stats: List[int] = field(default_factory=lambda: [0, 0, 0, 0])
    exceptions: Dict[int, str] = field(default_factory=dict)  # error code -> message (EXCEPTION_METADATA_KEY)


# QueryException.QUERY_EXECUTION_ERROR (common/exception/QueryException.java) and BROKER_GATHER_ERROR_CODE
QUERY_EXECUTION_ERROR_CODE = 200
BROKER_GATHER_ERROR_CODE = 300


class ServerQueryExecutor:
    """ServerQueryExecutorV1Impl.processQuery (core/query/executor/ServerQueryExecutorV1Impl.java:118-176) over the
    GPU plan maker: the inter-segment plan over this server's segments, its combined block turned into a response; an
    exception becomes an exception-only response."""

    def __init__(self, ctx: E.Context):
        self.plan_maker = E.InstancePlanMakerImplV2(ctx)

    def process_query(self, broker_request: dict, segments: Sequence[E.IndexSegment]) -> InstanceResponse:
        try:
            blk = self.plan_maker.make_inter_segment_plan(segments, broker_request).execute()
        except Exception as e:  # noqa: BLE001 -- surfaced to the broker as a processing exception
            return InstanceResponse(exceptions={QUERY_EXECUTION_ERROR_CODE: str(e)})
        resp = InstanceResponse(stats=blk.stats.as_list())
        if broker_request.get("group_by"):
            resp.group_by = blk.trimmed if blk.trimmed is not None else [{} for _ in broker_request["aggregations"]]
        else:
            resp.aggregation = list(blk.get_aggregation_result())
        return resp

    processQuery = process_query


@dataclass
class GroupByResult:
    group: List[str]
    value: str


@dataclass
class AggregationResult:
    function: str
    value: Optional[str] = None
    group_by_result: Optional[List[GroupByResult]] = None
    group_by_columns: Optional[List[str]] = None


@dataclass
class QueryProcessingException:
    error_code: int
    message: str


@dataclass
class BrokerResponseNative:
    aggregation_results: List[AggregationResult] = field(default_factory=list)
    num_docs_scanned: int = 0
    num_entries_scanned_in_filter: int = 0
    num_entries_scanned_post_filter: int = 0
    total_docs: int = 0
    processing_exceptions: List[QueryProcessingException] = field(default_factory=list)


class BrokerReduceService:
    """core/query/reduce/BrokerReduceService.java:62-256 for aggregation and aggregation-group-by requests."""

    def reduce_on_data_table(self, broker_request: dict, responses: Dict[str, InstanceResponse]) -> BrokerResponseNative:
        out = BrokerResponseNative()
        if not responses:
            return out  # BrokerResponseNative.EMPTY_RESULT
        live = {}
        for server, resp in responses.items():
            if resp is None:
                continue
            if isinstance(resp, (bytes, bytearray)):  # a serialized DataTable (pinot_amd/datatable.py)
                from .datatable import datatable_to_response
                resp = datatable_to_response(broker_request, bytes(resp))
            if resp.aggregation is None and resp.group_by is None:  # schema-less: exception metadata only
                for code, msg in resp.exceptions.items():
                    out.processing_exceptions.append(QueryProcessingException(int(code), msg))
                continue
            out.num_docs_scanned += int(resp.stats[0])
            out.num_entries_scanned_in_filter += int(resp.stats[1])
            out.num_entries_scanned_post_filter += int(resp.stats[2])
            out.total_docs += int(resp.stats[3])
            live[server] = resp
        aggs = broker_request["aggregations"]
        try:
            if broker_request.get("group_by"):
                out.aggregation_results = self._reduce_group_by(broker_request, list(live.values()))
            else:
                for i, a in enumerate(aggs):
                    v = _reduce(a["fn"], [r.aggregation[i] for r in live.values()])
                    out.aggregation_results.append(AggregationResult(function_name(a), _format(a["fn"], v)))
        except Exception as e:  # noqa: BLE001 -- BrokerReduceService.java:183-189
            out.processing_exceptions.append(QueryProcessingException(BROKER_GATHER_ERROR_CODE, str(e)))
        return out

    reduceOnDataTable = reduce_on_data_table

    @staticmethod
    def _reduce_group_by(broker_request: dict, responses: List[InstanceResponse]) -> List[AggregationResult]:
        """reduceGroupByOperators (combineTwoValues per key, then reduce per key) + renderAggregationGroupByResult
        (top N per function; AggregationGroupByOperatorService.java:93-129, :197-244)."""
        gb = broker_request["group_by"]
        cols = list(gb["columns"])
        top_n = gb.get("top_n", 10)
        results = []
        for i, a in enumerate(broker_request["aggregations"]):
            fn = a["fn"]
            merged: Dict[str, object] = {}
            for r in responses:
                for k, v in r.group_by[i].items():
                    merged[k] = _combine_two(fn, merged.get(k), v)
            reduced = {k: _reduce(fn, [v]) for k, v in merged.items() if v is not None}
            # MinMaxPriorityQueue of size topN: MIN functions ascending, others descending; ties in queue order
            # (arbitrary in the reference; broken by the group string here so the output is deterministic)
            best = sorted(reduced.items(), key=lambda kv: (kv[1] if fn == "min" else -kv[1], kv[0]))[:top_n]
            rows = [GroupByResult(k.split("\t", len(cols) - 1), _format(fn, v)) for k, v in best]
            results.append(AggregationResult(function_name(a), None, rows, cols))
        return results
