"""Golden routing matchers (direct / fanout / topic).

Reference: chana-mq-server/.../engine/QueueMatcher.scala
  * trait QueueMatcher {subscribe, unsubscribe, lookup}      :11-27
  * DirectMatcher: exact key -> subscribers                   :29-48
  * FanoutMatcher: every subscriber, key ignored              :50-66
  * TrieMatcher: words split on regex "\\." (Java split drops trailing
    empty strings), '*' matches exactly one word             :68-601
    The reference treats '#' literally (getBranches :261-263); SURVEY §7.4
    recommends standard AMQP '#' (zero or more words).  ``hash_wildcard``
    selects: True (default, AMQP 0-9-1 semantics) or False (reference parity).

These are the host golden models the HIP route kernels (K6) are tested against.
The GPU path stores the same word tokenisation (``split_words``).
"""


def split_words(key: str):
    """Java ``String.split("\\\\.")`` semantics (trailing empty strings dropped)."""
    if key == "":
        return [""]
    parts = key.split(".")
    while parts and parts[-1] == "":
        parts.pop()
    return parts


def topic_match(pattern: str, key: str, hash_wildcard: bool = True) -> bool:
    pw = split_words(pattern)
    kw = split_words(key)
    return words_match(pw, kw, hash_wildcard)


def words_match(pw, kw, hash_wildcard=True) -> bool:
    # dynamic programming over (pattern word, key word); O(|p|*|k|)
    np_, nk = len(pw), len(kw)
    reach = [False] * (nk + 1)
    reach[0] = True
    for i in range(np_):
        w = pw[i]
        nxt = [False] * (nk + 1)
        if hash_wildcard and w == "#":
            acc = False
            for j in range(nk + 1):
                acc = acc or reach[j]
                nxt[j] = acc
        else:
            for j in range(nk):
                if reach[j] and (w == "*" or w == kw[j]):
                    nxt[j + 1] = True
        reach = nxt
    return reach[nk]


class QueueMatcher:
    def subscribe(self, key, subscriber):
        raise NotImplementedError

    def unsubscribe(self, key, subscriber):
        raise NotImplementedError

    def lookup(self, key):
        raise NotImplementedError


class DirectMatcher(QueueMatcher):
    def __init__(self):
        self.table = {}

    def subscribe(self, key, sub):
        self.table.setdefault(key, set()).add(sub)

    def unsubscribe(self, key, sub):
        s = self.table.get(key)
        if s is not None:
            s.discard(sub)
            if not s:
                del self.table[key]

    def unsubscribe_all(self, sub):
        for k in list(self.table):
            self.unsubscribe(k, sub)

    def lookup(self, key):
        return set(self.table.get(key, ()))

    def bindings(self):
        return [(k, s) for k, subs in self.table.items() for s in subs]


class FanoutMatcher(QueueMatcher):
    def __init__(self):
        self.subs = {}  # sub -> set(keys)

    def subscribe(self, key, sub):
        self.subs.setdefault(sub, set()).add(key)

    def unsubscribe(self, key, sub):
        ks = self.subs.get(sub)
        if ks is not None:
            ks.discard(key)
            if not ks:
                del self.subs[sub]

    def unsubscribe_all(self, sub):
        self.subs.pop(sub, None)

    def lookup(self, key):
        return set(self.subs)

    def bindings(self):
        return [(k, s) for s, ks in self.subs.items() for k in ks]


class TopicMatcher(QueueMatcher):
    """Pattern list + DP match.  (The reference's CAS trie exists only to be
    lock-free inside one actor — SURVEY §5.2 — so a flat list is the honest
    golden model; the device kernel is the fast path.)"""

    def __init__(self, hash_wildcard=True):
        self.patterns = {}  # pattern -> set(subs)
        self.hash_wildcard = hash_wildcard

    def subscribe(self, key, sub):
        self.patterns.setdefault(key, set()).add(sub)

    def unsubscribe(self, key, sub):
        s = self.patterns.get(key)
        if s is not None:
            s.discard(sub)
            if not s:
                del self.patterns[key]

    def unsubscribe_all(self, sub):
        for k in list(self.patterns):
            self.unsubscribe(k, sub)

    def lookup(self, key):
        kw = split_words(key)
        out = set()
        for p, subs in self.patterns.items():
            if words_match(split_words(p), kw, self.hash_wildcard):
                out |= subs
        return out

    def bindings(self):
        return [(k, s) for k, subs in self.patterns.items() for s in subs]


def make_matcher(ex_type: str, hash_wildcard=True) -> QueueMatcher:
    """direct/fanout as named; topic, headers and any other type route via topic
    (ExchangeEntity.scala:149-154,211-216)."""
    if ex_type == "direct":
        return DirectMatcher()
    if ex_type == "fanout":
        return FanoutMatcher()
    return TopicMatcher(hash_wildcard)
