"""Query shapes exercised by the parity tests (small corpora the oracle
finishes in well under a second)."""
from workload import Word, build_query, config_two_term, config3_queries


def kinds(num_docs=20000, seed=1):
    N = num_docs
    out = [
        config_two_term(N, docs_to_get=50, seed=seed),
        build_query("three_word", [Word("a", 0.3), Word("b", 0.2), Word("c", 0.25)], N, seed=seed + 1),
        build_query("quoted_phrase", [Word("new", 0.3), Word("york", 0.3), Word("city", 0.3), Word("pizza", 0.2)],
                    N, seed=seed + 2, quoted=(0, 2)),
        build_query("negative", [Word("a", 0.4), Word("b", 0.3), Word("c", 0.1, sign=ord('-'))], N, seed=seed + 3),
        build_query("synonyms", [Word("car", 0.2, synonyms=(0.1,)), Word("cheap", 0.3)], N, seed=seed + 4),
        build_query("wiki_halfstop", [Word("time", 0.3, wiki=1), Word("enough", 0.4, wiki=1),
                                      Word("love", 0.3, wiki=1)], N, seed=seed + 5, half_stop_bigram=1),
        build_query("piped", [Word("a", 0.3), Word("b", 0.3, piped=1), Word("c", 0.3)], N, seed=seed + 6),
        build_query("single", [Word("solo", 0.05)], N, seed=seed + 7, docs_to_get=10),
        build_query("five_word", [Word(f"w{i}", 0.35) for i in range(5)], N, seed=seed + 8, docs_to_get=20),
        build_query("dense", [Word("x", 0.9), Word("y", 0.8)], N, seed=seed + 9, docs_to_get=200),
    ]
    out += config3_queries(N, docs_to_get=100, seed=seed + 10)[:4]
    return out
