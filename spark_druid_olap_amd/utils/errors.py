"""Exception types (``sd/DruidDataSourceException.scala:20``)."""


class DruidDataSourceException(RuntimeError):
    """Raised for engine / datasource failures surfaced to SQL clients."""


class QueryCancelled(DruidDataSourceException):
    """A query was cancelled (client cancel, deadline, or session close)."""


class QueryTimeout(QueryCancelled):
    """A query exceeded its deadline (``spark.sparklinedata.druid.query.timeout.ms``)."""
