"""A small PQL subset compiler producing the BrokerRequest fields this hot path consumes.

It covers exactly what the per-segment aggregation / group-by path reads from a BrokerRequest
(pinot-common/src/thrift/request.thrift): the aggregation list, the group-by columns + topN and the
filter query tree.  Encodings follow the reference compiler:
  * comparisons become RANGE strings, e.g. ``col > 5`` -> "(5\t\t*)", ``col <= 5`` -> "(*\t\t5]"
    (pinot-common/.../pql/parsers/pql2/ast/ComparisonPredicateAstNode.java:85-121);
  * BETWEEN a AND b -> "[a\t\tb]" (BetweenPredicateAstNode.java:55);
  * = / <> / != / IN / NOT IN -> EQ / NEQ / IN / NOT_IN with the literal values as strings;
  * chains of the same boolean operator are one AND/OR node with all children, in source order;
  * GROUP BY without TOP defaults to topN 10 (SelectAstNode.java:33,135-139).

The output is a plain dict (the "query spec") shared by the product path and the test oracle:
  {"aggregations": [{"fn": "sum", "column": "m"}, ...],
   "group_by": {"columns": [...], "top_n": 10} | None,
   "filter": None | {"op": "AND"|"OR", "children": [...]}
                   | {"op": "EQ"|"NEQ"|"IN"|"NOT_IN"|"RANGE", "column": c, "values": [str, ...]}}
"""
import re

_TOKEN = re.compile(r"\s*(?:(?P<num>-?\d+(?:\.\d+)?(?:[eE][-+]?\d+)?)|(?P<str>'(?:[^']|'')*'|\"(?:[^\"])*\")|"
                    r"(?P<op><=|>=|<>|!=|=|<|>|\(|\)|,|\*)|(?P<id>[A-Za-z_][A-Za-z0-9_.$]*))")

AGG_FUNCTIONS = ("count", "sum", "min", "max", "avg", "countmv", "summv", "minmv", "maxmv", "avgmv")
# distinctcount / minmaxrange / percentileNN (AggregationFunctionFactory.java:84-107): aggregation-only requests
EXT_FUNCTIONS = ("distinctcount", "distinctcounthll", "fasthll", "minmaxrange", "percentile50", "percentile90", "percentile95",
                 "percentile99", "percentileest50", "percentileest90", "percentileest95", "percentileest99")
# the same functions over every value of a multi-value column (AggregationFunctionFactory.java:48-58)
EXT_MV_FUNCTIONS = ("distinctcountmv", "distinctcounthllmv", "minmaxrangemv") + tuple(
    "percentile%dmv" % p for p in (50, 90, 95, 99)) + tuple("percentileest%dmv" % p for p in (50, 90, 95, 99))
EXT_FUNCTIONS = EXT_FUNCTIONS + EXT_MV_FUNCTIONS


class PqlError(ValueError):
    pass


def _tokenize(s):
    pos, out = 0, []
    s = s.strip()
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m or m.end() == pos:
            raise PqlError("cannot tokenize at: " + s[pos:pos + 20])
        pos = m.end()
        if m.group("num") is not None:
            out.append(("lit", m.group("num")))
        elif m.group("str") is not None:
            v = m.group("str")
            out.append(("lit", v[1:-1].replace("''", "'")))
        elif m.group("op") is not None:
            out.append(("op", m.group("op")))
        else:
            out.append(("id", m.group("id")))
    return out


class _P:
    def __init__(self, toks):
        self.t = toks
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def kw(self, word):
        k, v = self.peek()
        return k == "id" and v.upper() == word

    def take(self, kind=None, val=None):
        k, v = self.peek()
        if kind and k != kind:
            raise PqlError("expected %s got %r" % (kind, v))
        if val and (v is None or v.upper() != val.upper()):
            raise PqlError("expected %s got %r" % (val, v))
        self.i += 1
        return v

    def literal(self):
        k, v = self.peek()
        if k not in ("lit", "id"):
            raise PqlError("expected literal, got %r" % (v,))
        self.i += 1
        return v

    # predicate := and ( OR and )*
    def predicate(self):
        kids = [self.conj()]
        while self.kw("OR"):
            self.take()
            kids.append(self.conj())
        return kids[0] if len(kids) == 1 else {"op": "OR", "children": kids}

    def conj(self):
        kids = [self.primary()]
        while self.kw("AND"):
            self.take()
            kids.append(self.primary())
        return kids[0] if len(kids) == 1 else {"op": "AND", "children": kids}

    def primary(self):
        if self.peek() == ("op", "("):
            self.take()
            p = self.predicate()
            self.take("op", ")")
            return p
        col = self.take("id")
        k, v = self.peek()
        if k == "op" and v in ("=", "<>", "!="):
            self.take()
            lit = self.literal()
            return {"op": "EQ" if v == "=" else "NEQ", "column": col, "values": [lit]}
        if k == "op" and v in ("<", "<=", ">", ">="):
            self.take()
            lit = self.literal()
            rng = {"<": "(*\t\t%s)", "<=": "(*\t\t%s]", ">": "(%s\t\t*)", ">=": "[%s\t\t*)"}[v] % lit
            return {"op": "RANGE", "column": col, "values": [rng]}
        if self.kw("BETWEEN"):
            self.take()
            lo = self.literal()
            self.take("id", "AND")
            hi = self.literal()
            return {"op": "RANGE", "column": col, "values": ["[%s\t\t%s]" % (lo, hi)]}
        neg = False
        if self.kw("NOT"):
            self.take()
            neg = True
        if self.kw("IN"):
            self.take()
            self.take("op", "(")
            vals = [self.literal()]
            while self.peek() == ("op", ","):
                self.take()
                vals.append(self.literal())
            self.take("op", ")")
            return {"op": "NOT_IN" if neg else "IN", "column": col, "values": vals}
        raise PqlError("unsupported predicate near %r" % (v,))


def compile(pql: str) -> dict:  # noqa: A001 - mirrors Pql2Compiler.compileToBrokerRequest
    p = _P(_tokenize(pql))
    p.take("id", "SELECT")
    aggs = []
    while True:
        fn = p.take("id").lower()
        if fn not in AGG_FUNCTIONS and fn not in EXT_FUNCTIONS:
            raise PqlError("unsupported aggregation function " + fn)
        p.take("op", "(")
        k, v = p.peek()
        if (k, v) == ("op", "*"):
            p.take()
            col = "*"
        else:
            col = p.take("id")
        p.take("op", ")")
        aggs.append({"fn": fn, "column": col})
        if p.peek() == ("op", ","):
            p.take()
            continue
        break
    p.take("id", "FROM")
    table = p.take("id")
    filt = None
    group = None
    top = None
    while p.peek()[0] is not None:
        if p.kw("WHERE"):
            p.take()
            filt = p.predicate()
        elif p.kw("GROUP"):
            p.take()
            p.take("id", "BY")
            cols = [p.take("id")]
            while p.peek() == ("op", ","):
                p.take()
                cols.append(p.take("id"))
            group = cols
        elif p.kw("TOP"):
            p.take()
            top = int(p.literal())
        else:
            raise PqlError("unexpected token %r" % (p.peek()[1],))
    return {"table": table, "aggregations": aggs,
            "group_by": {"columns": group, "top_n": 10 if top is None else top} if group else None,
            "filter": filt}
