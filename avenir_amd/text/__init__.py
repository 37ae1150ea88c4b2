"""Text processing and text models (reference P/text)."""
from .models import (Doc2Vec, EmbeddingTextRankSumm, LatentDirichletAllocation, LatentSemSumm, NonNegMatFactSumm,
                     SumBasicSumm, Summarizer, TermFreqSumm, TextNaiveBayes, TextRankSumm, Word2Vec,
                     max_marginal_relevance, nmf, pagerank)
from .preprocess import (BiGram, DocSentences, NGram, TextPreProcessor, TfIdf, TriGram, Vocabulary,
                         WordVectorContainer, clean_tokens, cosine_similarity_matrix, doc_term_matrix, porter_stem,
                         split_sentences, tfidf_matrix)
