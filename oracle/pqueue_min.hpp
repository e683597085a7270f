// oracle/pqueue_min.hpp — TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
//
// Restatement of pqueue-1.3.1.1 `Data.PQueue.Min.MinQueue` (stack.yaml:21 pins
// pqueue-1.3.1.1; its sources are NOT in /root/reference — this follows the
// published binomial-heap algorithm as summarised in SURVEY.md Appendix B).
// It is used by the oracle's "pqueue" mode only, to reproduce TimedT's tie
// order among equal-timestamp events (Event's Ord compares _timestamp only,
// src/Control/TimeWarp/Timed/TimedT.hs:100-104).  PARITY UNPINNED: no reference
// test or fixture pins equal-timestamp pop order.
//
//   MinQueue = Empty | MinQueue n xmin forest      (global min held outside)
//   insert x : x <= xmin  -> x becomes min, old min carried into the forest
//              otherwise  -> x carried into the forest
//   incr t   : binary-counter carry; at a Cons t', Skip (incr (joinBin t t'))
//   joinBin  : t1 on top iff root t1 <= root t2 (incoming tree wins ties)
//   minView  : return xmin; new min = lowest-rank root among minimal roots;
//              its children are merged back rank by rank (placed at a Skip,
//              joinBin existing-first + carry at a Cons).
//   toList   = toAscList (repeated minView);  fromList = foldr insert empty
#pragma once
#include <cstddef>
#include <vector>

template <class T, class LEq>
class PQueueMin {
    struct Node {
        T x;
        std::vector<Node*> kids;  // kids[i] is the rank-i child
    };

  public:
    explicit PQueueMin(LEq le = LEq()) : le_(le) {}
    ~PQueueMin() { clear(); }
    PQueueMin(const PQueueMin&) = delete;
    PQueueMin& operator=(const PQueueMin&) = delete;

    bool empty() const { return n_ == 0; }
    size_t size() const { return n_; }
    const T& top() const { return min_; }

    void clear() {
        for (Node* t : forest_) free_tree(t);
        forest_.clear();
        n_ = 0;
    }

    // insert' le x (MinQueue n x' ts)
    void insert(const T& x) {
        if (n_ == 0) {
            min_ = x;
            n_ = 1;
            return;
        }
        if (le_(x, min_)) {
            Node* t = tip(min_);
            min_ = x;
            incr(t, 0);
        } else {
            incr(tip(x), 0);
        }
        ++n_;
    }

    // minView: returns the held minimum and extracts the next one from the forest.
    T pop() {
        T out = min_;
        --n_;
        if (n_ > 0) extract_heap();
        return out;
    }

    // toList (= toAscList) followed by clear.
    std::vector<T> drain_ascending() {
        std::vector<T> v;
        v.reserve(n_);
        while (n_ > 0) v.push_back(pop());
        return v;
    }

    // fromList = foldr insert empty : the LAST element is inserted first.
    void from_list(const std::vector<T>& v) {
        clear();
        for (size_t i = v.size(); i-- > 0;) insert(v[i]);
    }

  private:
    Node* tip(const T& x) {
        Node* n = new Node;
        n->x = x;
        return n;
    }
    void free_tree(Node* t) {
        if (!t) return;
        for (Node* k : t->kids) free_tree(k);
        delete t;
    }
    // joinBin le t1 t2 : t1 on top iff root t1 <= root t2
    Node* join(Node* t1, Node* t2) {
        if (le_(t1->x, t2->x)) {
            t1->kids.push_back(t2);
            return t1;
        }
        t2->kids.push_back(t1);
        return t2;
    }
    // incr le t f, with f the forest from rank k upward
    void incr(Node* t, size_t k) {
        for (;;) {
            if (k >= forest_.size()) {  // Nil -> Cons t Nil
                forest_.push_back(t);
                return;
            }
            if (!forest_[k]) {  // Skip f -> Cons t f
                forest_[k] = t;
                return;
            }
            Node* t2 = forest_[k];  // Cons t' f -> Skip (incr (joinBin t t') f)
            forest_[k] = nullptr;
            t = join(t, t2);
            ++k;
        }
    }
    // extractHeap / extractBin: the recursion compares on the way back up, so
    // a lower-rank root replaces the candidate unless the candidate is strictly
    // smaller (`lt` = not (b <= a)).  Phase 1 finds that root; phase 2 performs
    // the incrExtract / incrExtract' rebuild from rank m-1 down to rank 0.
    void extract_heap() {
        int m = -1;
        for (int k = (int)forest_.size() - 1; k >= 0; --k) {
            Node* t = forest_[k];
            if (!t) continue;
            if (m < 0 || !lt(forest_[m]->x, t->x)) m = k;
        }
        Node* w = forest_[m];
        forest_[m] = nullptr;  // Extract x ts (Skip f)
        for (int k = m - 1; k >= 0; --k) {
            Node* kc = w->kids[k];
            if (!forest_[k]) {
                forest_[k] = kc;  // incrExtract: Cons kChild ts
            } else {
                Node* t = forest_[k];  // incrExtract': Skip (incr (t `joinBin` kChild) ts)
                forest_[k] = nullptr;
                incr(join(t, kc), (size_t)k + 1);
            }
        }
        while (!forest_.empty() && !forest_.back()) forest_.pop_back();
        min_ = w->x;
        delete w;
    }
    bool lt(const T& a, const T& b) const { return !le_(b, a); }

    LEq le_;
    T min_{};
    size_t n_ = 0;
    std::vector<Node*> forest_;
};
