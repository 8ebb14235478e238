"""Hot-path constants, restated from the reference's config.py (lines cited per block).

Importing this module has no side effects (the reference's config.py creates directories
and log handlers on import, config.py:16-27; that is deliberately not mirrored)."""

TYPES = ["clicks", "carts", "orders"]                       # config.py:35
TYPE2ID = {"clicks": 0, "carts": 1, "orders": 2}           # config.py:36

MIN_TIME_TO_NEXT = -24 * 60 * 60                            # config.py:41
MAX_TIME_TO_NEXT = 24 * 60 * 60                             # config.py:42
MAP_MAX_TIME_TO_NEXT = {                                    # config.py:43-49
    "click_to_click": 12 * 60 * 60,
    "click_to_cart_or_buy": MAX_TIME_TO_NEXT,
    "cart_to_cart": MAX_TIME_TO_NEXT,
    "cart_to_buy": MAX_TIME_TO_NEXT,
    "buy_to_buy": MAX_TIME_TO_NEXT,
}
OPTIM_ROWS_POLARS_GROUPBY = 100_000_000                     # config.py:52
MAX_ROWS_POLARS_GROUPBY = 300_000_000                       # config.py:53
MIN_COUNT_TO_SAVE = {                                       # config.py:56-62
    "click_to_click": 10,
    "click_to_cart_or_buy": 5,
    "cart_to_cart": 2,
    "cart_to_buy": 2,
    "buy_to_buy": 2,
}
MIN_COUNT_IN_PART = {"click_to_click": 2, "click_to_cart_or_buy": 2}   # config.py:63
MAX_CO_EVENT_PAIRS_TO_SAVE_DISK = 300_000_000               # config.py:64
CO_EVENTS_TO_COUNT = [                                      # config.py:67-73
    "click_to_click",
    "click_to_cart_or_buy",
    "cart_to_cart",
    "cart_to_buy",
    "buy_to_buy",
]
RETRIEVE_N_LAST_CLICKS = 99                                 # config.py:76-79
RETRIEVE_N_LAST_CARTS = 99
RETRIEVE_N_LAST_ORDERS = 99
RETRIEVE_N_MOST_FREQUENT = 99
MAP_NAME_COUNT_TYPE = {                                     # config.py:81-88
    "click_to_click": (0, [0]),
    "click_to_cart_or_buy": (0, [1, 2]),
    "cart_to_cart": (1, [1]),
    "cart_to_buy": (1, [2]),
    "buy_to_buy": (2, [2]),
}
RETRIEVAL_FIRST_N_CO_COUNTS = {                             # config.py:90-96
    "click_to_click": 10,
    "click_to_cart_or_buy": 10,
    "cart_to_cart": 20,
    "cart_to_buy": 20,
    "buy_to_buy": 20,
}
RETRIEVAL_CO_COUNTS_TO_JOIN = list(CO_EVENTS_TO_COUNT)      # config.py:98-104

KEEP_TOP_K = 20                                             # config.py:31
W2VEC_SEARCH_SIMILAR_FOR_FIRST_N_AIDS = 600_000             # config.py:109
W2VEC_K = 20                                                # config.py:124
W2VEC_VECTOR_SIZE = 100                                     # config.py:120

N_ITEMS_OTTO = 1_855_603                                    # OTTO catalogue (dataset card)
# threshold of count_co_events.py:131 (literal in the reference)
CLICK_FILTER_ROWS = 100_000_000
